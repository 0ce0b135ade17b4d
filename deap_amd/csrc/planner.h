// Part of gpeval.hip's single translation unit (included there once, in
// order, inside the library's anonymous namespace): the launch planner — case
// tiles and LDS budgets per core, plan() (cost sort, snake deal, tile groups)
// and the launches of each kernel family.
#pragma once
namespace {

int fast_k(const gpe_ctx* ctx) {
  return ctx->prec == GPE_PREC_F32 ? kFK32 : kFK;
}

// asm_k: the asm core's cases per lane (Launch::K), 0 for the C++ kernels
int cases_per_tile(const gpe_ctx* ctx, bool deep, int asm_k) {
  if (ctx->machine == GPE_MACHINE_F)
    return asm_k ? 64 * asm_k : deep ? 64 : 64 * fast_k(ctx);
  return 64;  // B: 64 words per tile
}

// the cases per lane of an asm launch: the fp32 cores, or the fp64 fast /
// deep / exact / typed core
int asm_core_k(const gpe_ctx* ctx, bool deep_core, bool exact, bool typed) {
  if (typed) return asmcore_typed::K;
  if (ctx->prec == GPE_PREC_F32 && !exact) return asmcore32::K;
  if (exact) return asmcore_exact::K;
  return deep_core ? asmcore_deep::K : asmcore::K;
}

// sdepth: the launch's stack slots per wave (F machine; default: the
// kernel's maximum, for capacity checks)
size_t lds_bytes(const gpe_ctx* ctx, bool deep, int sdepth = 0, int wpb = kWaves) {
  if (ctx->machine == GPE_MACHINE_F) {
    const int K = deep ? 1 : fast_k(ctx);
    const int D = sdepth > 0 ? sdepth : deep ? kDeepDepth : kFastDepth;
    const size_t el = ctx->prec == GPE_PREC_F32 ? sizeof(float) : sizeof(double);
    return (size_t)(ctx->nv + ctx->nt + wpb * D) * K * 64 * el;
  }
  const int D = deep ? kDeepDepth : kFastDepth;
  return (size_t)(ctx->nv + 1 + kWaves * D) * 64 * sizeof(uint32_t);
}

// the typed core's LDS: the case tile (+ labels) only
size_t lds_bytes_typed(const gpe_ctx* ctx) {
  return (size_t)(ctx->nv + ctx->nt) * asmcore_typed::K * 64 * sizeof(double);
}

// f_eval_asm's second tile buffer (AsmTask::dbuf): fp64, 16-byte aligned
// case rows (the LDS-DMA copies 16 bytes per lane), 1 KiB columns (K = 2)
bool asm_dbuf(const gpe_ctx* ctx, int K) {
  return ctx->asm_dbuf && ctx->prec == GPE_PREC_F64 && ctx->n_cases % 2 == 0 &&
         K * 64 * sizeof(double) == 1024;
}

size_t lds_bytes_asm(const gpe_ctx* ctx, int P, int wpb, int K, bool dbuf,
                     bool exact = false) {
  const bool f32 = !exact && ctx->prec == GPE_PREC_F32 && K == asmcore32::K;
  const size_t tile = f32 ? (size_t)(ctx->nv + ctx->nt) * K * 64 * sizeof(float)
                          : (size_t)(ctx->nv + ctx->nt) * K * 64 * sizeof(double) *
                                (dbuf ? 2 : 1);
  // (f_eval_asm's kTab: the exact cores' glibc tables are half the table
  // core's, which leaves room for a sixth program per wave on C4)
  const size_t table = f32 ? 0 : exact ? (size_t)asmcore_exact::GLIBC_LDS_BYTES : kTrigLdsBytes;
  return table + tile + (size_t)wpb * P * 128 * sizeof(double);
}

// B machine with at most 16 words of cases: lanes per program of the
// lane-packed kernel (b_eval_lanes), else 0.  GPE_B_LANES=0 disables.
int b_lane_group(const gpe_ctx* ctx) {
  if (ctx->machine != GPE_MACHINE_B || ctx->n_units > 16 || !ctx->b_lanes) return 0;
  int G = 1;
  while (G < ctx->n_units) G <<= 1;
  return G;
}

// Balance: programs sorted by length (descending) are dealt to waves in a
// snake order, so every wave's total work is about the mean.
int plan(gpe_ctx* ctx, Launch& L, const std::vector<int32_t>& progs, bool deep,
         bool is_asm, bool deep_core = false, bool typed = false, bool exact = false) {
  L.n_slots = 0;
  L.waves = 0;
  L.programs = (int64_t)progs.size();
  L.sdepth = 1;
  L.K = is_asm ? asm_core_k(ctx, deep_core, exact, typed) : 0;
  if (progs.empty()) {
    L.slot_prog.clear();         // (no stale slots of an earlier batch)
    return 0;
  }
  auto t_q = std::chrono::steady_clock::now();
  auto qlap = [&](const char* what) {
    if (!ctx->diag) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "  plan %s %.3f ms\n", what,
            std::chrono::duration<double, std::milli>(now - t_q).count());
    t_q = now;
  };
  const int64_t n = (int64_t)progs.size();
  // host threads over contiguous ranges of progs at pop 1M (the serial
  // passes below were 5-6 ms of C5's plan)
  const int nth = n >= 262144 ? host_threads() : 1;
  auto chunk = [&](int t, int64_t m) {
    return std::make_pair(m * t / nth, m * (t + 1) / nth);
  };
  // the launch's stack slots and the largest cost (the sort's buckets), in
  // one pass
  int64_t cmax = 0;
  {
    std::vector<int> td((size_t)nth, 1);
    std::vector<int64_t> tc((size_t)nth, 0);
    hostpool::par_run(nth, [&](int t) {
      const auto [a, b] = chunk(t, n);
      int d = 1;
      int64_t c = 0;
      for (int64_t r = a; r < b; ++r) {
        const size_t p = (size_t)progs[(size_t)r];
        d = std::max<int>(d, ctx->depth[p]);
        c = std::max<int64_t>(c, ctx->cost[p]);
      }
      td[(size_t)t] = d;
      tc[(size_t)t] = c;
    });
    L.sdepth = *std::max_element(td.begin(), td.end());
    cmax = *std::max_element(tc.begin(), tc.end());
  }
  // (the typed core: no per-program LDS; its tiny programs share each
  // staged tile — C5's is 59 KB — among more of them)
  const int pmax = typed ? ctx->typed_pmax : is_asm ? ctx->asm_pmax : 16;
  // the largest P (programs per wave: they share each staged tile) that
  // still leaves ~4 waves per block of the grid target busy
  const int64_t units0 = ctx->machine == GPE_MACHINE_F ? ctx->n_cases : ctx->n_units;
  const int64_t tiles0 = std::max<int64_t>(
      1, (units0 + cases_per_tile(ctx, deep, L.K) - 1) /
             cases_per_tile(ctx, deep, L.K));
  const int64_t want = 4 * ctx->target_blocks;
  L.P = (int)std::max<int64_t>(
      1, std::min<int64_t>(pmax, n * std::min<int64_t>(tiles0, 65535) / want));
  // asm: the largest P whose LDS still admits two blocks per CU (16 waves,
  // the VGPR limit); the accumulators take P KiB per wave
  // (deep core: smaller blocks, three of them per CU — its VGPRs allow 3
  // waves per SIMD)
  // C++ F kernels: 8 waves share a staged tile when two such blocks still
  // fit a CU's LDS (wide case tiles: C5's 57 variables)
  int wpb = typed ? ctx->typed_waves
                  : is_asm ? (deep_core ? ctx->asm_deep_waves : ctx->asm_waves) : kWaves;
  if (!is_asm && ctx->machine == GPE_MACHINE_F && ctx->f_waves == 8 &&
      lds_bytes(ctx, deep, L.sdepth, 8) <= 80 * 1024)
    wpb = 8;
  const size_t lds_cap = deep_core ? 48 * 1024 : (size_t)ctx->asm_lds_kb * 1024;
  if (!is_asm && b_lane_group(ctx)) L.P = 64 / b_lane_group(ctx);  // a lane group each
  L.dbuf = false;
  if (is_asm && !typed) {
    auto fit = [&](bool db) {
      int P = L.P;
      while (P > 1 && lds_bytes_asm(ctx, P, wpb, L.K, db, exact) > lds_cap) --P;
      return P;
    };
    // the second tile buffer costs the accumulators' LDS: taken while it
    // leaves at least 4 programs per wave (or all of them) and at most 2
    // fewer than one buffer (C4: P 7 -> 5 measured 0.7 % faster; the
    // trig-leaf tiles, 31 columns, would drop P 4 -> 1)
    const int p1 = fit(false);
    const int p2 = asm_dbuf(ctx, L.K) ? fit(true) : 0;
    L.dbuf = p2 > 0 && p2 + 2 >= p1 && (p2 >= 4 || p2 == p1) &&
             lds_bytes_asm(ctx, p2, wpb, L.K, true, exact) <= lds_cap;
    L.P = L.dbuf ? p2 : p1;
  }
  const int64_t W = (n + L.P - 1) / L.P;
  L.wpb = wpb;
  const int64_t Wb = (W + wpb - 1) / wpb * wpb;
  L.waves = Wb;
  L.n_slots = Wb * L.P;
  // balance by estimated cost, not length: sin/cos nodes dominate, and the
  // waves of a block meet at a barrier every tile.  Stable descending
  // counting sort (costs are small integers).
  qlap("shape");
  const std::vector<int32_t>& cost = ctx->cost;
  // the slots are dealt straight into the launch's own pinned staging (an
  // asynchronous copy from a pageable vector has the runtime pin it first;
  // run_common syncs before the next plan reuses the staging); the host keeps
  // a copy only of the asm launches' slots, which run_common reads back
  int32_t* slots = (int32_t*)pinned_buf(&L.h_pin, &L.h_pin_cap,
                                        (size_t)L.n_slots * sizeof(int32_t));
  if (!slots) return fail(ctx, GPE_E_HIP, "hipHostMalloc (launch plan)");
  if ((!is_asm && b_lane_group(ctx)) || (typed && n >= (1 << 17))) {
    // the lane-packed B kernel (at most 16 words of cases), and the typed
    // core's large launches: programs in program order, no cost sort — the
    // sort's three passes over a million programs cost more than the balance
    // saved (C3 at pop 1M: kernel 0.141 -> 0.228 ms, the evaluate's device
    // calls 2.27-2.67 -> 1.83-2.34 ms, scripts/r05_bsort.sh; C5: kernel
    // 3.66 -> 3.76 ms, device calls 5.83-6.11 -> 5.33-5.47 ms,
    // scripts/r05_typed_sort.sh — 64 tiny programs per wave average out)
    hostpool::par_run(nth, [&](int t) {
      const auto [a, b] = chunk(t, L.n_slots);
      for (int64_t r = a; r < b; ++r) slots[r] = r < n ? progs[(size_t)r] : -1;
    });
    goto slots_done;
  }
  {
  std::vector<int32_t>& order = ctx->pl_order;
  order.resize(progs.size());
  if (nth > 1 && cmax < 65536) {
    // stable descending counting sort: per-thread histograms, bucket-major
    // offsets (thread t's items of a bucket after threads < t's), scatter
    const size_t nb = (size_t)cmax + 1;
    std::vector<int64_t> hist((size_t)nth * nb, 0);
    hostpool::par_run(nth, [&](int t) {
      const auto [a, b] = chunk(t, n);
      int64_t* h = hist.data() + (size_t)t * nb;
      for (int64_t r = a; r < b; ++r) ++h[(size_t)(cmax - cost[(size_t)progs[(size_t)r]])];
    });
    int64_t run = 0;
    for (size_t c = 0; c < nb; ++c)
      for (int t = 0; t < nth; ++t) {
        int64_t& h = hist[(size_t)t * nb + c];
        const int64_t k = h;
        h = run;
        run += k;
      }
    hostpool::par_run(nth, [&](int t) {
      const auto [a, b] = chunk(t, n);
      int64_t* h = hist.data() + (size_t)t * nb;
      for (int64_t r = a; r < b; ++r) {
        const int32_t p = progs[(size_t)r];
        order[(size_t)h[(size_t)(cmax - cost[(size_t)p])]++] = p;
      }
    });
  } else if (cmax < (int64_t)16 * 1024 * 1024) {
    std::vector<int64_t>& start = ctx->pl_start;
    start.assign((size_t)cmax + 2, 0);
    for (int32_t p : progs) ++start[(size_t)(cmax - cost[p]) + 1];
    for (size_t c = 1; c < start.size(); ++c) start[c] += start[c - 1];
    for (int32_t p : progs) order[(size_t)start[(size_t)(cmax - cost[p])]++] = p;
  } else {
    order = progs;
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
      return cost[a] > cost[b];
    });
  }
  if (ctx->diag) fprintf(stderr, "  plan cmax %lld\n", (long long)cmax);
  qlap("order");
  {
    // the snake deal, by wave: slot (wave wv, round) holds order[round * W
    // + pos], pos = wv on even rounds and W - 1 - wv on odd ones; each thread
    // writes its own waves' slots (threads dealing ranges of `order` wrote
    // one another's cache lines: 6 ms at C5's P)
    const int64_t P = L.P;
    const int mix = (is_asm && !typed) ? ctx->deal_mix : 0;
    hostpool::par_run(nth, [&](int t) {
      const auto [a, b] = chunk(t, Wb);
      for (int64_t wv = a; wv < b; ++wv)
        for (int64_t round = 0; round < P; ++round) {
          const int64_t pos = (round & 1) ? (W - 1 - wv) : wv;
          const int64_t r = round * W + pos;
          slots[wv * P + round] = wv < W && r < n ? order[(size_t)r] : -1;
        }
      if (mix == 1)         // (the valid slots are a prefix: reverse just it)
        for (int64_t wv = a | 1; wv < b; wv += 2) {
          int32_t* w = slots + wv * P;
          int64_t m = 0;
          while (m < P && w[m] >= 0) ++m;
          std::reverse(w, w + m);
        }
      if (mix == 2)         // wave wv starts at band wv mod P (rotated prefix)
        for (int64_t wv = a; wv < b; ++wv) {
          int32_t* w = slots + wv * P;
          int64_t m = 0;
          while (m < P && w[m] >= 0) ++m;
          if (m > 1) std::rotate(w, w + (wv % m), w + m);
        }
    });
  }
  }
slots_done:
  if (&L == &ctx->fasm || &L == &ctx->dasm)
    L.slot_prog.assign(slots, slots + L.n_slots);
  else
    L.slot_prog.clear();
  qlap("slots");
  const int64_t units = ctx->machine == GPE_MACHINE_F ? ctx->n_cases : ctx->n_units;
  const int64_t per = cases_per_tile(ctx, deep, L.K);
  L.n_tiles = std::max<int64_t>(1, (units + per - 1) / per);
  const int64_t blocks_y = Wb / wpb;
  const int64_t target_blocks = typed    ? ctx->typed_target_blocks
                                : is_asm ? ctx->asm_target_blocks
                                         : ctx->target_blocks;
  int64_t groups = std::max<int64_t>(1, target_blocks / std::max<int64_t>(1, blocks_y));
  // at least min_group_tiles tiles per group (a block's fixed work — its
  // first tile's staging, the accumulators, the closing reduction — stays
  // small against its tiles when the cases are few: a rank of a sharded run)
  if (is_asm && ctx->min_group_tiles > 0)
    groups = std::min<int64_t>(groups, std::max<int64_t>(8, L.n_tiles / ctx->min_group_tiles));
  // XCD-aware: workgroups go to the 8 XCDs round-robin by linear id (x
  // fastest), so with groups a multiple of 8 all blocks of a tile group
  // share one XCD's L2 and stream the same tiles from it (groups = 6 on
  // C4 fetched 14x the bytes of groups = 8 from beyond L2)
  if (L.n_tiles >= 8 && groups >= 4) groups = std::max<int64_t>(8, groups / 8 * 8);
  groups = std::min<int64_t>(groups, L.n_tiles);
  groups = std::min<int64_t>(groups, 65535);
  L.tiles_per_group = (int)((L.n_tiles + groups - 1) / groups);
  L.groups = (int)((L.n_tiles + L.tiles_per_group - 1) / L.tiles_per_group);
  if (ensure(ctx, &L.d_slot_prog, &L.slot_cap, (size_t)L.n_slots)) return GPE_E_HIP;
  HIPCHK(hipMemcpyAsync(L.d_slot_prog, slots, (size_t)L.n_slots * sizeof(int32_t),
                        hipMemcpyHostToDevice, ctx->stream));
  qlap("h2d");
  if (ensure(ctx, &L.d_part, &L.part_cap, (size_t)L.groups * L.n_slots * 2))
    return GPE_E_HIP;
  qlap("part");
  return 0;
}

template <int K, int D, int MODE, typename R, bool EXACT = false>
int launch_f(gpe_ctx* ctx, Launch& L, bool deep, unsigned long long* err,
             uint32_t* flags) {
  if (L.n_slots == 0) return 0;
  Task a{};
  a.code = ctx->d_code;
  a.off = ctx->d_off;
  a.slot_prog = L.d_slot_prog;
  a.n_slots = L.n_slots;
  a.P = L.P;
  a.X = ctx->d_X;
  a.nv = ctx->nv;
  a.terms = ctx->d_terms;
  a.nt = ctx->nt;
  a.n_cases = ctx->n_cases;
  a.n_units = ctx->n_cases;
  a.n_tiles = L.n_tiles;
  a.tiles_per_group = L.tiles_per_group;
  a.part = L.d_part;
  a.case_out = ctx->case_on ? ctx->d_case_out : nullptr;
  a.first_err = err;
  a.flags = flags;
  a.sdepth = std::min(L.sdepth, D);
  size_t lds = lds_bytes(ctx, deep, a.sdepth, L.wpb);
  if (EXACT && lds + kGlibcLdsDoubles * sizeof(double) <= 160 * 1024) {
    a.gtab_lds = 1;
    lds += kGlibcLdsDoubles * sizeof(double);
  }
  auto kern = f_eval<K, D, MODE, R, EXACT>;
  HIPCHK(hipFuncSetAttribute((const void*)kern,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  dim3 grid((unsigned)L.groups, (unsigned)(L.waves / L.wpb));
  hipLaunchKernelGGL(kern, grid, dim3(64 * L.wpb), lds, ctx->stream, a);
  HIPCHK(hipGetLastError());
  return 0;
}

int launch_asm(gpe_ctx* ctx, Launch& L, unsigned long long* err,
               uint32_t* flags, bool deep_core = false, bool exact = false) {
  if (L.n_slots == 0) return 0;
  AsmTask a{};
  a.code = exact ? ctx->d_acode_x : ctx->d_acode;
  a.start = exact ? ctx->d_astart_x : ctx->d_astart;
  a.slot_prog = L.d_slot_prog;
  a.n_slots = L.n_slots;
  a.P = L.P;
  a.X = (const double*)ctx->d_X;
  a.nv = ctx->nv;
  a.terms = (const double*)ctx->d_terms;
  a.nt = ctx->nt;
  a.n_cases = ctx->n_cases;
  a.n_tiles = L.n_tiles;
  a.tiles_per_group = L.tiles_per_group;
  a.part = L.d_part;
  a.case_out = ctx->case_on ? ctx->d_case_out : nullptr;
  a.first_err = err;
  a.flags = flags;
  a.redo = ctx->d_redo;
  a.redo_count = ctx->d_redo_count;
  a.redo_list = ctx->d_redo_list;
  a.redo_list_cap = ctx->redo_list_cap;
  a.cst = ctx->d_cst;
  a.cst32 = ctx->d_cst32;
  a.diag = ctx->diag;
  a.redo_hi = deep_core ? std::min(ctx->redo_hi, ctx->redo_hi_deep) : ctx->redo_hi;
  if (exact) {                 // flags: lanes past the core's glibc range
    a.redo = ctx->d_redo2;
    a.redo_count = ctx->d_redo2_count;
    a.redo_hi = asmcore_exact::EXACT_REDO_HI;
    a.cst = ctx->d_cst_exact;
  }
  a.dbuf = L.dbuf ? 1 : 0;
  const size_t lds = lds_bytes_asm(ctx, L.P, L.wpb, L.K, L.dbuf, exact);
  const bool f32 = ctx->prec == GPE_PREC_F32;
  auto kern = exact ? (deep_core ? f_eval_asm<false, true, true> : f_eval_asm<false, false, true>)
              : deep_core ? (f32 ? f_eval_asm<true, true> : f_eval_asm<false, true>)
                          : (f32 ? f_eval_asm<true, false> : f_eval_asm<false, false>);
  HIPCHK(hipFuncSetAttribute((const void*)kern,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  dim3 grid((unsigned)L.groups, (unsigned)(L.waves / L.wpb));
  hipLaunchKernelGGL(kern, grid, dim3(64 * L.wpb), lds, ctx->stream, a);
  HIPCHK(hipGetLastError());
  return 0;
}

int launch_asm_typed(gpe_ctx* ctx, Launch& L) {
  if (L.n_slots == 0) return 0;
  AsmTask a{};
  a.code = ctx->d_acode_t;
  a.start = ctx->d_astart_t;
  a.slot_prog = L.d_slot_prog;
  a.n_slots = L.n_slots;
  a.P = L.P;
  a.X = (const double*)ctx->d_X;
  a.nv = ctx->nv;
  a.terms = (const double*)ctx->d_terms;
  a.nt = ctx->nt;
  a.n_cases = ctx->n_cases;
  a.n_tiles = L.n_tiles;
  a.tiles_per_group = L.tiles_per_group;
  a.part = L.d_part;
  const size_t lds = lds_bytes_typed(ctx);
  HIPCHK(hipFuncSetAttribute((const void*)f_eval_asm_typed,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  dim3 grid((unsigned)L.groups, (unsigned)(L.waves / L.wpb));
  hipLaunchKernelGGL(f_eval_asm_typed, grid, dim3(64 * L.wpb), lds, ctx->stream, a);
  HIPCHK(hipGetLastError());
  return 0;
}

template <int D>
int launch_b(gpe_ctx* ctx, Launch& L, bool deep) {
  const int G = b_lane_group(ctx);
  if (L.n_slots == 0) return 0;
  Task a{};
  a.code = ctx->d_code;
  a.off = ctx->d_off;
  a.slot_prog = L.d_slot_prog;
  a.n_slots = L.n_slots;
  a.P = L.P;
  a.X = ctx->d_X;
  a.nv = ctx->nv;
  a.terms = ctx->d_terms;
  a.nt = 1;
  a.n_cases = ctx->n_cases;
  a.n_units = ctx->n_units;
  a.n_tiles = L.n_tiles;
  a.tiles_per_group = L.tiles_per_group;
  a.part = L.d_part;
  const size_t lds = lds_bytes(ctx, deep);
  dim3 grid((unsigned)L.groups, (unsigned)(L.waves / kWaves));
  if (G) {                                   // tiny case sets: lane-packed
    auto kern = b_eval_lanes<D>;
    HIPCHK(hipFuncSetAttribute((const void*)kern,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, grid, dim3(kBlock), lds, ctx->stream, a, G);
    HIPCHK(hipGetLastError());
    return 0;
  }
  auto kern = b_eval<D>;
  HIPCHK(hipFuncSetAttribute((const void*)kern,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, grid, dim3(kBlock), lds, ctx->stream, a);
  HIPCHK(hipGetLastError());
  return 0;
}

int launch_reduce(gpe_ctx* ctx, Launch& L, double* hi, double* lo) {
  if (L.n_slots == 0) return 0;
  const unsigned blocks = (unsigned)((L.n_slots + 255) / 256);
  hipLaunchKernelGGL(reduce_groups, dim3(blocks), dim3(256), 0, ctx->stream,
                     L.d_part, L.n_slots, L.groups, L.d_slot_prog, hi, lo);
  HIPCHK(hipGetLastError());
  return 0;
}

}  // namespace
