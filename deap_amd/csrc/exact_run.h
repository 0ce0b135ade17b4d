// Part of gpeval.hip's single translation unit (included there once, in
// order, inside the library's anonymous namespace): the glibc-exact pass — the C++
// pair pass for (program, tile)s past the exact core's range, the exact cores'
// launches (run_exact_asm) and the exact-int host evaluator (run_exact_host).
#pragma once
namespace {

// The asm core's left-out (program, tile) pairs: sorted on the device,
// evaluated one wave each by f_eval_pairs, then added to the programs' sums
// in tile order.
int redo_pairs(gpe_ctx* ctx, uint32_t cnt, double* hi, double* lo,
               unsigned long long* err, uint32_t* flags, bool count = true,
               int64_t max_runs = -1) {
  // radix sort of the 64-bit keys (program << 32 | tile): the order
  // std::sort gives, whatever order the atomics appended them in
  size_t tmp_bytes = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, ctx->d_redo_list,
                                           ctx->d_redo_list, (int)cnt, 0, 64,
                                           ctx->stream));
  if (ensure(ctx, &ctx->d_sort_tmp, &ctx->sort_tmp_cap, tmp_bytes)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_pair_sorted, &ctx->pair_sorted_cap, cnt)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_pair_part, &ctx->pair_part_cap, (size_t)cnt * 2)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_pair_off, &ctx->pair_off_cap, cnt)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_pair_nruns, &ctx->pair_nruns_cap, 1)) return GPE_E_HIP;
  HIPCHK(hipcub::DeviceRadixSort::SortKeys(ctx->d_sort_tmp, tmp_bytes, ctx->d_redo_list,
                                           ctx->d_pair_sorted, (int)cnt, 0, 64,
                                           ctx->stream));
  HIPCHK(hipMemsetAsync(ctx->d_pair_nruns, 0, sizeof(uint32_t), ctx->stream));
  hipLaunchKernelGGL(pair_runs, dim3((cnt + 255) / 256), dim3(256), 0, ctx->stream,
                     (const uint64_t*)ctx->d_pair_sorted, (int64_t)cnt, ctx->d_pair_off,
                     ctx->d_pair_nruns);
  HIPCHK(hipGetLastError());
  Task a{};
  a.code = ctx->d_code;
  a.off = ctx->d_off;
  a.X = ctx->d_X;
  a.nv = ctx->nv;
  a.terms = ctx->d_terms;
  a.nt = ctx->nt;
  a.n_cases = ctx->n_cases;
  a.n_units = ctx->n_cases;
  a.case_out = ctx->case_on ? ctx->d_case_out : nullptr;
  a.first_err = err;
  a.flags = flags;
  const bool f32 = ctx->prec == GPE_PREC_F32;
  // the tiles of the core whose (program, tile) pairs these are: the fp32
  // core's, or the exact core's (fp64)
  const int K = f32 ? asmcore32::K : asmcore_exact::K;
  // stack slots for programs of either asm core
  constexpr int kPairDepth = asmcore_deep::D;
  const size_t lds = (size_t)(ctx->nv + ctx->nt + kPairDepth) * K * 64 *
                     (f32 ? sizeof(float) : sizeof(double));
  // fp32: the C++ fp32 interpreter; fp64 (the exact core's pairs): the C++
  // exact interpreter (glibc_trig_k)
  auto kern = f32 ? f_eval_pairs<asmcore32::K, kPairDepth, float>
                  : f_eval_pairs<asmcore_exact::K, kPairDepth, double>;
  HIPCHK(hipFuncSetAttribute((const void*)kern,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3(cnt), dim3(64), lds, ctx->stream, a,
                     (const uint64_t*)ctx->d_pair_sorted, ctx->d_pair_part);
  HIPCHK(hipGetLastError());
  // one wave per program (at most max_runs of them, and at most cnt)
  const int64_t runs_cap = std::min<int64_t>(cnt, max_runs < 0 ? ctx->n_prog : max_runs);
  hipLaunchKernelGGL(add_pairs, dim3((unsigned)runs_cap), dim3(64), 0, ctx->stream,
                     (const uint64_t*)ctx->d_pair_sorted, (int64_t)cnt,
                     (const int64_t*)ctx->d_pair_off, (const uint32_t*)ctx->d_pair_nruns,
                     (const double*)ctx->d_pair_part, hi, lo);
  HIPCHK(hipGetLastError());
  if (count) {
    uint32_t runs = 0;
    HIPCHK(hipMemcpyAsync(&runs, ctx->d_pair_nruns, sizeof(uint32_t),
                          hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->redo_programs = (int64_t)runs;
  }
  return 0;
}

// The exact core over the flagged programs `rx` (their entries already
// cleared): translate them for it, run, reduce; programs it flags (a lane
// past its glibc range) are cleared again and appended to `rest` for the
// C++ exact kernels.
int run_exact_asm(gpe_ctx* ctx, const std::vector<int32_t>& rx, double* hi,
                  double* lo, unsigned long long* err, uint32_t* flags,
                  std::vector<int32_t>& rest,
                  const std::vector<int32_t>& rxd = std::vector<int32_t>()) {
  const int64_t n_prog = ctx->n_prog;
  // the flagged programs' threaded code for the exact cores (rx: D = 5;
  // rxd: the deep one), translated on the device (no host copy of the
  // programs)
  std::vector<uint8_t> cls((size_t)n_prog, 0);
  for (const std::vector<int32_t>* v : {&rx, &rxd})
    for (int32_t i : *v)
      if (i < 0 || i >= n_prog) return fail(ctx, GPE_E_STATE, "exact core: program index out of range");
  for (int32_t i : rx) cls[(size_t)i] = 1;
  for (int32_t i : rxd) cls[(size_t)i] = 2;
  XlateTabs T{};
  T.tab[0] = T.tab[2] = ctx->d_jump_asm_exact;
  T.ids[0] = T.ids[2] = kIds;
  T.tab[1] = ctx->d_jump_asm_exact_deep;
  T.ids[1] = kIdsExactDeep;
  int rc0 = translate_device(ctx, &cls, T, false, false, &ctx->d_acode_x, &ctx->acode_x_cap,
                             &ctx->d_astart_x, &ctx->astart_x_cap);
  if (rc0) return rc0;
  if (ensure(ctx, &ctx->d_redo2, &ctx->redo2_cap, (size_t)n_prog)) return GPE_E_HIP;
  HIPCHK(hipMemsetAsync(ctx->d_redo2, 0, (size_t)n_prog * sizeof(uint32_t), ctx->stream));
  HIPCHK(hipMemsetAsync(ctx->d_redo2_count, 0, sizeof(uint32_t), ctx->stream));
  int rc;
  // the main core's block geometry (the exact core's constants live in
  // registers: its VGPRs allow 4 waves per SIMD); a grid target of its own
  // (GPE_XASM_TARGET_BLOCKS)
  const int64_t keep = ctx->asm_target_blocks;
  ctx->asm_target_blocks = ctx->xasm_target_blocks;
  rc = plan(ctx, ctx->redo_xasm, rx, false, true, false, false, true);
  ctx->asm_target_blocks = keep;
  if (rc) return rc;
  if ((rc = plan(ctx, ctx->redo_xasm_deep, rxd, false, true, true, false, true))) return rc;
  if ((rc = launch_asm(ctx, ctx->redo_xasm, err, flags, false, true))) return rc;
  if ((rc = launch_asm(ctx, ctx->redo_xasm_deep, err, flags, true, true))) return rc;
  if ((rc = launch_reduce(ctx, ctx->redo_xasm, hi, lo))) return rc;
  if ((rc = launch_reduce(ctx, ctx->redo_xasm_deep, hi, lo))) return rc;
  uint32_t cnt = 0;
  HIPCHK(hipMemcpyAsync(&cnt, ctx->d_redo2_count, sizeof(uint32_t), hipMemcpyDeviceToHost,
                        ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  ctx->redo_exact_cpp = cnt;
  if (!cnt) return 0;
  // the (program, tile) pairs with a lane past the core's range: the C++
  // exact interpreter, added to the programs' sums (as the fp32 pair pass)
  if (cnt <= ctx->redo_list_cap)
    return redo_pairs(ctx, cnt, hi, lo, err, flags, false,
                      (int64_t)(rx.size() + rxd.size()));
  std::vector<uint32_t> flagged((size_t)n_prog);
  HIPCHK(hipMemcpy(flagged.data(), ctx->d_redo2, n_prog * sizeof(uint32_t),
                   hipMemcpyDeviceToHost));
  std::vector<int32_t> again;
  for (const std::vector<int32_t>* v : {&rx, &rxd})
    for (int32_t i : *v)
      if (flagged[(size_t)i]) again.push_back(i);
  if (ensure(ctx, &ctx->d_redo_progs, &ctx->redo_progs_cap, again.size())) return GPE_E_HIP;
  HIPCHK(hipMemcpy(ctx->d_redo_progs, again.data(), again.size() * sizeof(int32_t),
                   hipMemcpyHostToDevice));
  hipLaunchKernelGGL(clear_entries, dim3((unsigned)((again.size() + 255) / 256)),
                     dim3(256), 0, ctx->stream, ctx->d_redo_progs, (int64_t)again.size(),
                     err, flags);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(ctx->stream));
  rest.insert(rest.end(), again.begin(), again.end());
  return 0;
}

// host twins of two_sum / dd_add (the library is built with
// -ffp-contract=off: the same roundings as the device's)
void h_two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
  if (!std::isfinite(s)) e = 0.0;
}
void h_dd_add(double& hi, double& lo, double bhi, double blo) {
  double s, e;
  h_two_sum(hi, bhi, s, e);
  e = e + (lo + blo);
  const double h = s + e;
  double l = e - (h - s);
  if (!std::isfinite(h)) l = 0.0;
  hi = h;
  lo = l;
}

// The host half of the exact pass (bigint_host.h): exact-list entries `ents`
// evaluated over this context's cases with unbounded ints — f_eval_exact's
// per-case term, first error and flags, summed in exact_rows_sum's order —
// written into the device result arrays (and per-case outputs).
// run_exact_host's results: rec[5 i ..] = (program, hi bits, lo bits, first
// error, flags)
__global__ __launch_bounds__(256) void scatter_results(const uint64_t* rec, int64_t m,
                                                       double* hi, double* lo,
                                                       unsigned long long* err,
                                                       uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t* r = rec + 5 * i;
  const int64_t p = (int64_t)r[0];
  hi[p] = __longlong_as_double((long long)r[1]);
  lo[p] = __longlong_as_double((long long)r[2]);
  err[p] = (unsigned long long)r[3];
  flags[p] = (uint32_t)r[4];
}

int run_exact_host(gpe_ctx* ctx, int mode, const std::vector<int64_t>& ents, double* hi,
                   double* lo, unsigned long long* err, uint32_t* flags) {
  if (ents.empty()) return 0;
  const int64_t nc = ctx->n_cases;
  const int nvu = ctx->nv_user, nt = ctx->nt;
  if (!ctx->ex_hcases) {                 // the cases, once per gpe_set_cases
    ctx->ex_hX.resize((size_t)nvu * nc);
    ctx->ex_hT.resize((size_t)nt * nc);
    if (nvu) HIPCHK(hipMemcpy(ctx->ex_hX.data(), ctx->d_X, ctx->ex_hX.size() * sizeof(double),
                              hipMemcpyDeviceToHost));
    if (nt) HIPCHK(hipMemcpy(ctx->ex_hT.data(), ctx->d_terms, ctx->ex_hT.size() * sizeof(double),
                             hipMemcpyDeviceToHost));
    ctx->ex_hcases = true;
  }
  const hbig::Rows rows{ctx->ex_h_words.data(), ctx->ex_h_woff.data(),
                        ctx->ex_h_woff.empty() ? 0 : (int64_t)ctx->ex_h_woff.size() - 1};
  const double* X = ctx->ex_hX.data();
  const double* terms = ctx->ex_hT.data();
  const auto t_h0 = std::chrono::steady_clock::now();
  std::vector<double> term((size_t)nc);
  // the programs' results, written to the device in one copy and one
  // scatter kernel at the end: (prog, hi bits, lo bits, err, flags) each
  std::vector<uint64_t> rec;
  rec.reserve(ents.size() * 5);
  for (const int64_t ent : ents) {
    const int prog = ctx->ex_h_progs[(size_t)ent];
    const uint32_t* W = ctx->ex_h_code.data() + ctx->ex_h_off[(size_t)ent];
    const int nch = (int)std::min<int64_t>(256, std::max<int64_t>(1, nc / 64));
    std::vector<unsigned long long> cerr((size_t)nch, ~0ull);
    std::vector<uint32_t> cfl((size_t)nch, 0), cbad((size_t)nch, 0);
    hostpool::par_run(nch, [&](int ch) {
      const int64_t c0 = nc * ch / nch, c1 = nc * (ch + 1) / nch;
      for (int64_t c = c0; c < c1; ++c) {
        hbig::Num T;
        uint32_t e = hbig::E_NONE;
        auto xv = [&](uint32_t v) { return (int)v < nvu ? X[(int64_t)v * nc + c] : 0.0; };
        try {                            // (no exception may leave a pool thread)
          if (!hbig::run(W, rows, xv, T, e)) {
            cbad[(size_t)ch] = 1;
            return;
          }
        } catch (const std::bad_alloc&) {
          cbad[(size_t)ch] = 2;
          return;
        }
        double t = 0.0;
        if (mode == GPE_MODE_MSE && !e) {
          double dlt = hbig::to_f(T, e);
          for (int q = 0; q < nt; ++q) dlt = dlt - terms[(int64_t)q * nc + c];
          if (!e) {
            t = dlt * dlt;
            uint32_t fl = 0;
            const bool fin = std::isfinite(dlt);
            if (!fin) fl |= GPE_FLAG_NONFINITE_TERM;
            if (t != t) fl |= GPE_FLAG_NAN_TERM;
            if (std::isinf(t)) fl |= GPE_FLAG_INF_TERM;
            if (fin && std::isinf(t)) e = GPE_ERR_OVERFLOW;
            cfl[(size_t)ch] |= fl;
          }
        } else if (!e) {
          t = hbig::truth(T) == (terms[c] != 0.0) ? 1.0 : 0.0;
        }
        if (e) cerr[(size_t)ch] = std::min(cerr[(size_t)ch], ((unsigned long long)c << 2) | e);
        term[(size_t)c] = t;
      }
    });
    for (const uint32_t b : cbad) {
      if (b == 2) return fail(ctx, GPE_E_INVALID, "exact program: out of memory for its ints");
      if (b) return fail(ctx, GPE_E_INVALID, "exact program: opcode outside the exact set");
    }
    unsigned long long e = ~0ull;
    uint32_t fl = 0;
    for (int ch = 0; ch < nch; ++ch) {
      e = std::min(e, cerr[(size_t)ch]);
      fl |= cfl[(size_t)ch];
    }
    // exact_rows_sum: 256 strided double-double partials, then a fixed tree
    double sh[256], sl[256];
    for (int th = 0; th < 256; ++th) {
      double h = 0.0, l = 0.0;
      for (int64_t c = th; c < nc; c += 256) h_dd_add(h, l, term[(size_t)c], 0.0);
      sh[th] = h;
      sl[th] = l;
    }
    for (int m = 128; m >= 1; m >>= 1)
      for (int th = 0; th < m; ++th) h_dd_add(sh[th], sl[th], sh[th + m], sl[th + m]);
    uint64_t bh, bl;
    memcpy(&bh, &sh[0], 8);
    memcpy(&bl, &sl[0], 8);
    rec.insert(rec.end(), {(uint64_t)prog, bh, bl, (uint64_t)e, (uint64_t)fl});
    if (ctx->case_on)
      HIPCHK(hipMemcpy(ctx->d_case_out + (size_t)prog * nc, term.data(), nc * sizeof(double),
                       hipMemcpyHostToDevice));
  }
  if (ensure(ctx, &ctx->d_exh_rec, &ctx->exh_rec_cap, rec.size())) return GPE_E_HIP;
  uint64_t* d_rec = ctx->d_exh_rec;
  HIPCHK(hipMemcpyAsync(d_rec, rec.data(), rec.size() * sizeof(uint64_t),
                        hipMemcpyHostToDevice, ctx->stream));
  const int64_t m = (int64_t)ents.size();
  hipLaunchKernelGGL(scatter_results, dim3((unsigned)((m + 255) / 256)), dim3(256), 0,
                     ctx->stream, (const uint64_t*)d_rec, m, hi, lo, err, flags);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(ctx->stream));   // (rec is pageable host memory)
  ctx->ex_host_ms += std::chrono::duration<double, std::milli>(
                         std::chrono::steady_clock::now() - t_h0).count();
  return 0;
}

// The exact pass: the listed programs again, with Python-int semantics
// (f_eval_exact), their entries cleared first; rows in chunks of at most
// 64 MiB, summed per program in a fixed order.  Programs whose ints the
// device's 1088 bits cannot hold (an int constant past them, or a case the
// device ended with E_RANGE) are evaluated again on the host
// (run_exact_host: unbounded ints, the reference's semantics).
int run_exact(gpe_ctx* ctx, int mode, double* hi, double* lo,
              unsigned long long* err, uint32_t* flags) {
  const int64_t n = ctx->n_exact, nc = ctx->n_cases;
  if (nc <= 0) return 0;
  HIPCHK(hipEventRecord(ctx->ev_redo[0], ctx->stream));
  if (n > 0) {
    hipLaunchKernelGGL(clear_entries, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ctx->stream, (const int32_t*)ctx->d_ex_progs, n, err, flags);
    HIPCHK(hipGetLastError());
  }
  const int64_t chunk = std::max<int64_t>(
      1, std::min<int64_t>({std::max<int64_t>(n, 1), 65535, ((int64_t)64 << 20) / (nc * 8)}));
  if (n > 0 && ensure(ctx, &ctx->d_ex_rows, &ctx->ex_rows_cap, (size_t)(chunk * nc)))
    return GPE_E_HIP;
  for (int64_t i0 = 0; i0 < n; i0 += chunk) {
    const int64_t m = std::min(chunk, n - i0);
    hipLaunchKernelGGL(f_eval_exact, dim3((unsigned)((nc + 255) / 256), (unsigned)m),
                       dim3(256), 0, ctx->stream, (const uint32_t*)ctx->d_ex_code,
                       (const int64_t*)ctx->d_ex_off, (const int32_t*)ctx->d_ex_progs, i0,
                       (const uint32_t*)ctx->d_ex_ints, (const double*)ctx->d_X, ctx->nv,
                       (const double*)ctx->d_terms, ctx->nt, nc, mode, ctx->d_ex_rows,
                       ctx->case_on ? ctx->d_case_out : nullptr, err, flags);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(exact_rows_sum, dim3((unsigned)m), dim3(256), 0, ctx->stream,
                       (const double*)ctx->d_ex_rows, nc, (const int32_t*)ctx->d_ex_progs,
                       i0, hi, lo);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(ctx->ev_redo[1], ctx->stream));
  HIPCHK(hipEventSynchronize(ctx->ev_redo[1]));
  float ms = 0.0f;
  HIPCHK(hipEventElapsedTime(&ms, ctx->ev_redo[0], ctx->ev_redo[1]));
  ctx->ms[0] += ms;
  ctx->ms[2] += ms;
  // the host half: programs with ints past the device's, and device
  // programs whose first error is the device's range end
  std::vector<int64_t> host = ctx->ex_host;
  if (n > 0) {
    std::vector<unsigned long long> e((size_t)ctx->n_prog);
    HIPCHK(hipMemcpy(e.data(), err, e.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < n; ++j) {
      const int64_t ent = ctx->ex_dev_index[(size_t)j];
      const unsigned long long v = e[(size_t)ctx->ex_h_progs[(size_t)ent]];
      if (v != ~0ull && (v & 3u) == GPE_ERR_XINT_RANGE) host.push_back(ent);
    }
  }
  ctx->ex_host_runs = (int64_t)host.size();
  ctx->ex_host_ms = 0.0;
  return run_exact_host(ctx, mode, host, hi, lo, err, flags);
}

}  // namespace
