// Part of gpeval.hip's single translation unit (included there once, in
// order, inside the library's anonymous namespace for device code): the device lexicase and tournament selection
// kernels that replay the reference's random stream.
#pragma once
namespace {

// ------------------------------------------------------- lexicase ----
// Device lexicase selection that replays the reference's random stream.
// selLexicase / selEpsilonLexicase / selAutomaticEpsilonLexicase
// (deap/tools/selection.py:214-320) draw with random.shuffle(cases) and
// random.choice(candidates); CPython's Random is MT19937
// (Modules/_randommodule.c genrand_uint32) and both calls reduce to
// _randbelow_with_getrandbits(n): k = n.bit_length(), r = genrand >> (32 - k)
// until r < n (random.py).  The kernel receives random.getstate()'s 624
// words + position, makes exactly the reference's draws in the reference's
// order, and returns the state after them, so that a seeded run selects the
// same individuals and the host's random stream continues where the
// reference's would.  One workgroup runs the k selections in order (they
// share the stream); lane 0 draws, the block filters the candidates.
constexpr int kLexBlock = 256;
constexpr int kMtN = 624, kMtM = 397;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  return y ^ (y >> 18);
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
// the genrand_uint32 twist, in place (lane 0 only: a rare fallback)
__device__ void mt_twist_serial(uint32_t* mt) {
  int kk = 0;
  for (; kk < kMtN - kMtM; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + kMtM]);
  for (; kk < kMtN - 1; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + kMtM - kMtN]);
  mt[kMtN - 1] = mt_mix(mt[kMtN - 1], mt[0], mt[kMtM - 1]);
}
// the same twist into a second buffer by the whole block: four phases, each
// reading only words the serial loop would have read at that point
__device__ void mt_twist_block(const uint32_t* cur, uint32_t* nxt, int tid) {
  for (int kk = tid; kk < kMtN - kMtM; kk += kLexBlock)            // [0, 227)
    nxt[kk] = mt_mix(cur[kk], cur[kk + 1], cur[kk + kMtM]);
  __syncthreads();
  for (int kk = kMtN - kMtM + tid; kk < 2 * (kMtN - kMtM); kk += kLexBlock)
    nxt[kk] = mt_mix(cur[kk], cur[kk + 1], nxt[kk + kMtM - kMtN]);  // [227, 454)
  __syncthreads();
  for (int kk = 2 * (kMtN - kMtM) + tid; kk < kMtN - 1; kk += kLexBlock)
    nxt[kk] = mt_mix(cur[kk], cur[kk + 1], nxt[kk + kMtM - kMtN]);  // [454, 623)
  __syncthreads();
  if (tid == 0) nxt[kMtN - 1] = mt_mix(cur[kMtN - 1], nxt[0], nxt[kMtM - 1]);
  __syncthreads();
}
struct MtState {
  uint32_t buf[2][kMtN];
  int cur, idx, next_ok;
};
__device__ uint32_t mt_next(MtState& m) {          // genrand_uint32
  if (m.idx >= kMtN) {
    if (m.next_ok) {
      m.cur ^= 1;
      m.next_ok = 0;
    } else {
      mt_twist_serial(m.buf[m.cur]);
    }
    m.idx = 0;
  }
  return mt_temper(m.buf[m.cur][m.idx++]);
}
__device__ uint32_t mt_randbelow(MtState& m, uint32_t n) {  // random.py
  if (n == 0) return 0;
  const int k = 32 - __builtin_clz(n);
  uint32_t r;
  do {
    r = mt_next(m) >> (32 - k);
  } while (r >= n);
  return r;
}

// block sum of an int64 (every thread gets it)
__device__ int64_t lex_block_sum(int64_t v, int64_t* red, int tid) {
  red[tid] = v;
  __syncthreads();
  for (int h = kLexBlock / 2; h > 0; h >>= 1) {
    if (tid < h) red[tid] += red[tid + h];
    __syncthreads();
  }
  const int64_t r = red[0];
  __syncthreads();
  return r;
}

// k-th smallest of vals[0..m) (no nan): the value whose rank interval
// [#less, #less-or-equal) holds k (O(m^2) rank counting: automatic-epsilon
// candidate sets are small)
__device__ double lex_kth(const double* vals, int64_t m, int64_t kth,
                          double* shv, int tid) {
  for (int64_t i = tid; i < m; i += kLexBlock) {
    const double v = vals[i];
    int64_t lt = 0, le = 0;
    for (int64_t j = 0; j < m; ++j) {
      lt += vals[j] < v;
      le += vals[j] <= v;
    }
    if (lt <= kth && kth < le) *shv = v;           // equal values: same value
  }
  __syncthreads();
  const double r = *shv;
  __syncthreads();
  return r;
}
// numpy.median of vals[0..m): nan if any is nan, else the middle value or
// the mean of the two middle values ((a + b) / 2, numpy's mean of two)
__device__ double lex_median(const double* vals, int64_t m, double* shv,
                             int64_t* red, int tid) {
  int64_t nans = 0;
  for (int64_t i = tid; i < m; i += kLexBlock) nans += vals[i] != vals[i];
  if (lex_block_sum(nans, red, tid)) return __builtin_nan("");
  if (m & 1) return lex_kth(vals, m, m / 2, shv, tid);
  const double a = lex_kth(vals, m, m / 2 - 1, shv, tid);
  const double b = lex_kth(vals, m, m / 2, shv, tid);
  return (a + b) / 2.0;
}

// ------------------------------------------------ device tournament ----
// selTournament (deap/tools/selection.py:51-69): k tournaments of tournsize
// aspirants, each aspirant random.choice(individuals) = _randbelow(n) =
// getrandbits(bits) resampled while >= n (random.py), i.e. one tempered
// MT19937 word per try.  tournament_draws (one block) replays the stream:
// every 624-word state is tempered in parallel, the accepted words (r < n)
// are numbered by a block scan and stored as draws in order, and the state
// (buffer + position just past the last word used) is written back.
__global__ __launch_bounds__(kLexBlock) void tournament_draws(uint32_t* state, int64_t n,
                                                              int64_t total,
                                                              int32_t* draws) {
  __shared__ uint32_t mt[2][kMtN];
  __shared__ int64_t scan[kLexBlock];
  __shared__ int stop_at;
  const int tid = threadIdx.x;
  for (int i = tid; i < kMtN; i += kLexBlock) mt[0][i] = state[i];
  int cur = 0;
  int idx = (int)state[kMtN];
  const int bits = 32 - __builtin_clz((uint32_t)n);
  int64_t done = 0;
  if (tid == 0) stop_at = -1;
  __syncthreads();
  while (done < total) {
    if (idx >= kMtN) {
      mt_twist_block(mt[cur], mt[cur ^ 1], tid);
      cur ^= 1;
      idx = 0;
    }
    for (int base = idx; base < kMtN && done < total; base += kLexBlock) {
      const int p = base + tid;
      uint32_t r = 0;
      int64_t acc = 0;
      if (p < kMtN) {
        r = mt_temper(mt[cur][p]) >> (32 - bits);
        acc = r < (uint64_t)n;
      }
      scan[tid] = acc;
      __syncthreads();
      for (int h = 1; h < kLexBlock; h <<= 1) {     // inclusive scan
        const int64_t v = tid >= h ? scan[tid - h] : 0;
        __syncthreads();
        scan[tid] += v;
        __syncthreads();
      }
      const int64_t pos = done + scan[tid] - acc;    // draw number of this word
      if (acc && pos < total) {
        draws[pos] = (int32_t)r;
        if (pos == total - 1) stop_at = p;           // the last word used
      }
      done += scan[kLexBlock - 1];
      __syncthreads();
    }
    if (done < total) idx = kMtN;
  }
  __syncthreads();
  if (total > 0) idx = stop_at + 1;
  for (int i = tid; i < kMtN; i += kLexBlock) state[i] = mt[cur][i];
  if (tid == 0) state[kMtN] = (uint32_t)idx;
}

// Fitness.__gt__ (deap/base.py:218-219): not (a.wvalues <= b.wvalues) in
// Python tuple order (the first unequal component decides)
__device__ __forceinline__ bool wvalues_gt(const double* a, const double* b, int nobj) {
  for (int o = 0; o < nobj; ++o) {
    if (a[o] == b[o]) continue;
    return !(a[o] <= b[o]);
  }
  return false;
}
// max(aspirants, key=fitness): the first of the greatest
__global__ void tournament_pick(const double* wv, int nobj, const int32_t* draws,
                                int64_t k, int ts, int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  const int32_t* a = draws + i * ts;
  int32_t best = a[0];
  for (int j = 1; j < ts; ++j)
    if (wvalues_gt(wv + (int64_t)a[j] * nobj, wv + (int64_t)best * nobj, nobj)) best = a[j];
  out[i] = best;
}
// the last run's fitness as weighted values: weight * (MSE: (hi + lo) / n,
// SSE / hits: hi).  n: the divisor on the device (a case-sharded run's
// all-reduced case count) or, if null, n_cases.  raises (MSE, builtin-sum
// modes): a program whose evaluation raises in the reference — first_err set,
// or (MSE) an fsum that overflows on finite terms — gets nan and sets
// *status: the reference never reaches selection with such a population.
__global__ void fitness_wvalues(const double* hi, const double* lo,
                                const unsigned long long* err, const uint32_t* flags,
                                int64_t n, int mse, int raises, const int64_t* d_cases,
                                double n_cases, double weight, double* wv,
                                uint32_t* status) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double div = d_cases ? (double)*d_cases : n_cases;
  const double sse = mse ? hi[i] + lo[i] : hi[i];
  const bool bad = raises && (err[i] != ~0ull ||
                              (mse && __builtin_isinf(sse) &&
                               !(flags[i] & GPE_FLAG_NONFINITE_TERM)));
  if (bad) {
    wv[i] = __builtin_nan("");
    atomicOr(status, 1u);
    return;
  }
  wv[i] = weight * (mse ? sse / div : sse);
}

__global__ void set_i64(int64_t* p, int64_t v) { *p = v; }

__global__ __launch_bounds__(kLexBlock) void lexicase_mt(
    const double* val, int64_t n, int64_t C, const uint8_t* maximise, int mode,
    double eps, uint32_t* state, int64_t k, int32_t* out, int64_t* status,
    double* scratch) {
  extern __shared__ uint32_t lex_lds[];
  const int64_t nw = (n + 31) / 32;
  uint32_t* cand = lex_lds;                          // [nw] candidate bits
  uint32_t* perm = lex_lds + nw;                     // [C] shuffled cases
  __shared__ MtState mt;
  __shared__ double red_v[kLexBlock];
  __shared__ int64_t red_i[kLexBlock];
  __shared__ int64_t sh_fail;
  __shared__ double sh_v;
  const int tid = threadIdx.x;
  for (int i = tid; i < kMtN; i += kLexBlock) mt.buf[0][i] = state[i];
  if (tid == 0) {
    mt.cur = 0;
    mt.idx = (int)state[kMtN];
    mt.next_ok = 0;
    sh_fail = -1;
  }
  __syncthreads();
  for (int64_t sel = 0; sel < k; ++sel) {
    // the next state block, in parallel, when this selection may reach it
    // (C - 1 shuffle draws and one choice, usually one word each)
    if (!mt.next_ok && mt.idx + 2 * C + 64 >= kMtN) {
      mt_twist_block(mt.buf[mt.cur], mt.buf[mt.cur ^ 1], tid);
      if (tid == 0) mt.next_ok = 1;
    }
    for (int64_t w = tid; w < nw; w += kLexBlock) {
      const int64_t left = n - w * 32;
      cand[w] = left >= 32 ? 0xffffffffu : ((1u << left) - 1u);
    }
    for (int64_t c = tid; c < C; c += kLexBlock) perm[c] = (uint32_t)c;
    __syncthreads();
    if (tid == 0)                                    // random.shuffle(cases)
      for (int64_t i = C - 1; i >= 1; --i) {
        const uint32_t j = mt_randbelow(mt, (uint32_t)(i + 1));
        const uint32_t a = perm[i];
        perm[i] = perm[j];
        perm[j] = a;
      }
    __syncthreads();
    int64_t count = n;
    for (int64_t t = 0; t < C && count > 1; ++t) {
      const int64_t c = perm[t];                     // cases.pop(0) order
      const bool mx = maximise[c] != 0;
      // Python's max/min over the candidates in order: the first value,
      // replaced only by strictly better ones (a leading nan stays)
      double best = mx ? -__builtin_inf() : __builtin_inf();
      int64_t first = INT64_MAX;
      for (int64_t w = tid; w < nw; w += kLexBlock) {
        uint32_t bits = cand[w];
        while (bits) {
          const int b = __builtin_ctz(bits);
          bits &= bits - 1;
          const int64_t i = w * 32 + b;
          const double v = val[i * C + c];
          if (i < first) first = i;
          if (!__builtin_isnan(v)) best = mx ? fmax(best, v) : fmin(best, v);
        }
      }
      red_v[tid] = best;
      red_i[tid] = first;
      __syncthreads();
      for (int h = kLexBlock / 2; h > 0; h >>= 1) {
        if (tid < h) {
          red_v[tid] = mx ? fmax(red_v[tid], red_v[tid + h])
                          : fmin(red_v[tid], red_v[tid + h]);
          red_i[tid] = min(red_i[tid], red_i[tid + h]);
        }
        __syncthreads();
      }
      double b = red_v[0];
      const double v0 = val[red_i[0] * C + c];
      __syncthreads();
      if (__builtin_isnan(v0)) b = v0;
      double lim = b;
      if (mode == 1) {
        lim = mx ? b - eps : b + eps;
      } else if (mode == 2) {
        // median absolute deviation of the candidates' values (numpy),
        // candidates compacted in index order into scratch[0..count)
        int64_t mine = 0;
        for (int64_t w = tid; w < nw; w += kLexBlock) mine += __builtin_popcount(cand[w]);
        red_i[tid] = mine;
        __syncthreads();
        if (tid == 0) {                              // exclusive scan
          int64_t acc = 0;
          for (int q = 0; q < kLexBlock; ++q) {
            const int64_t x = red_i[q];
            red_i[q] = acc;
            acc += x;
          }
        }
        __syncthreads();
        int64_t pos = red_i[tid];
        __syncthreads();
        for (int64_t w = tid; w < nw; w += kLexBlock) {
          uint32_t bits = cand[w];
          while (bits) {
            const int bb = __builtin_ctz(bits);
            bits &= bits - 1;
            scratch[pos++] = val[(w * 32 + bb) * C + c];
          }
        }
        __syncthreads();
        const double med = lex_median(scratch, count, &sh_v, red_i, tid);
        for (int64_t i = tid; i < count; i += kLexBlock)
          scratch[n + i] = __builtin_fabs(scratch[i] - med);
        __syncthreads();
        const double mad = lex_median(scratch + n, count, &sh_v, red_i, tid);
        lim = mx ? b - mad : b + mad;
      }
      int64_t keep = 0;
      for (int64_t w = tid; w < nw; w += kLexBlock) {
        uint32_t bits = cand[w], out_bits = bits;
        while (bits) {
          const int bb = __builtin_ctz(bits);
          bits &= bits - 1;
          const double v = val[(w * 32 + bb) * C + c];
          const bool ok = mode == 0 ? (v == lim) : (mx ? v >= lim : v <= lim);
          if (!ok) out_bits &= ~(1u << bb);
        }
        cand[w] = out_bits;
        keep += __builtin_popcount(out_bits);
      }
      count = lex_block_sum(keep, red_i, tid);
    }
    if (tid == 0) {                                  // random.choice
      if (count == 0) {
        sh_fail = sel;                               // IndexError there
      } else {
        int64_t r = mt_randbelow(mt, (uint32_t)count);
        int64_t pick = -1;
        for (int64_t w = 0; w < nw; ++w) {
          const int pc = __builtin_popcount(cand[w]);
          if (r < pc) {
            uint32_t bits = cand[w];
            for (int64_t q = 0; q < r; ++q) bits &= bits - 1;
            pick = w * 32 + __builtin_ctz(bits);
            break;
          }
          r -= pc;
        }
        out[sel] = (int32_t)pick;
      }
    }
    __syncthreads();
    if (sh_fail >= 0) break;
  }
  // the state after the draws: the current block and position (a
  // precomputed next block is only a cache)
  for (int i = tid; i < kMtN; i += kLexBlock) state[i] = mt.buf[mt.cur][i];
  if (tid == 0) {
    state[kMtN] = (uint32_t)mt.idx;
    *status = sh_fail;
  }
}

__global__ void clear_entries(const int32_t* progs, int64_t n,
                              unsigned long long* err, uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    err[progs[i]] = ~0ull;
    flags[progs[i]] = 0;
  }
}


// The exact pass (gpe_load_exact): list entries [i0, i0 + gridDim.y) of the
// exact programs, one case per thread; the per-case term (MSE: the squared
// error, as f_eval forms it from float(T); HITS_BOOL: the match) goes to
// row i - i0 of `rows` (and to case_out when a per-case run asked for it).
constexpr int kXintDepth = 32;
__global__ __launch_bounds__(256) void f_eval_exact(
    const uint32_t* code, const int64_t* off, const int32_t* progs, int64_t i0,
    const uint32_t* ints, const double* X, int nv, const double* terms, int nt,
    int64_t n_cases, int mode, double* rows, double* case_out,
    unsigned long long* first_err, uint32_t* flags) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t li = i0 + blockIdx.y;
  const int prog = progs[li];
  if (c >= n_cases) return;
  xint::Num T;
  uint32_t err = xint::E_NONE;
  auto xv = [&](uint32_t v) { return X[(int64_t)v * n_cases + c]; };
  xint::run<kXintDepth>(code + off[li], ints, xv, T, err);
  double term = 0.0;
  if (mode == GPE_MODE_MSE && !err) {
    // (f(x) - t0 - ...)**2: an int result converts to float first
    double dlt = xint::to_f(T, err);
    for (int q = 0; q < nt; ++q) dlt = dlt - terms[(int64_t)q * n_cases + c];
    if (!err) {
      term = dlt * dlt;
      uint32_t fl = 0;
      const bool fin = __builtin_isfinite(dlt);
      if (!fin) fl |= GPE_FLAG_NONFINITE_TERM;
      if (term != term) fl |= GPE_FLAG_NAN_TERM;
      if (__builtin_isinf(term)) fl |= GPE_FLAG_INF_TERM;
      if (fin && __builtin_isinf(term)) err = GPE_ERR_OVERFLOW;
      if (fl) atomicOr(&flags[prog], fl);
    }
  } else if (!err) {
    term = xint::truth(T) == (terms[c] != 0.0) ? 1.0 : 0.0;
  }
  // the case's first error (the evaluation order's first exception)
  if (err) atomicMin(&first_err[prog], ((unsigned long long)c << 2) | err);
  rows[blockIdx.y * n_cases + c] = term;
  if (case_out) case_out[(size_t)prog * n_cases + c] = term;
}

// Row sums of the exact pass in a fixed order: MSE as double-double (each
// thread a strided part, then a fixed tree), hit counts exactly.
__global__ __launch_bounds__(256) void exact_rows_sum(const double* rows, int64_t n_cases,
                                                      const int32_t* progs, int64_t i0,
                                                      double* hi, double* lo) {
  __shared__ double sh[256], sl[256];
  const double* r = rows + blockIdx.x * n_cases;
  double h = 0.0, l = 0.0;
  for (int64_t c = threadIdx.x; c < n_cases; c += 256) dd_add(h, l, r[c], 0.0);
  sh[threadIdx.x] = h;
  sl[threadIdx.x] = l;
  __syncthreads();
  for (int m = 128; m >= 1; m >>= 1) {
    if ((int)threadIdx.x < m) {
      double a = sh[threadIdx.x], b = sl[threadIdx.x];
      dd_add(a, b, sh[threadIdx.x + m], sl[threadIdx.x + m]);
      sh[threadIdx.x] = a;
      sl[threadIdx.x] = b;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int prog = progs[i0 + blockIdx.x];
    hi[prog] = sh[0];
    lo[prog] = sl[0];
  }
}

}  // namespace
