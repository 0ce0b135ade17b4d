// Part of gpeval.hip's single translation unit (included there once, in
// order, inside the library's anonymous namespace for device code): the C++ interpreters — the F machine
// (f_eval, fp64/fp32 cases) and the bit-sliced B machine (b_eval, b_eval_lanes).
#pragma once
namespace {

// ---------------------------------------------------------------- F ----
template <int K, typename R>
__device__ __forceinline__ void ld_tile(const R* base, uint32_t idx,
                                        int lane, R (&o)[K]) {
  const R* p = base + (size_t)idx * (K * 64) + lane;
#pragma unroll
  for (int k = 0; k < K; ++k) o[k] = p[k * 64];
}

template <int K, typename R>
__device__ __forceinline__ void st_tile(R* base, uint32_t idx, int lane,
                                        const R (&v)[K]) {
  R* p = base + (size_t)idx * (K * 64) + lane;
#pragma unroll
  for (int k = 0; k < K; ++k) p[k * 64] = v[k];
}

#define FOR_K _Pragma("unroll") for (int k = 0; k < K; ++k)

// one binary family: a = operand (stack / variable / constant), b = T
#define F_BIN(BASE, EXPR)                                      \
  case BASE + 0: {                                             \
    ld_tile<K>(stk, d, lane, o);                               \
    FOR_K {                                                    \
      const R a = o[k], b = T[k];                              \
      T[k] = (EXPR);                                           \
    }                                                          \
    break;                                                     \
  }                                                            \
  case BASE + 1: {                                             \
    ld_tile<K>(xs, x, lane, o);                                \
    FOR_K {                                                    \
      const R a = o[k], b = T[k];                              \
      T[k] = (EXPR);                                           \
    }                                                          \
    break;                                                     \
  }                                                            \
  case BASE + 2: {                                             \
    const R c = (R)dbits(W[i], W[i + 1]);                      \
    i += 2;                                                    \
    FOR_K {                                                    \
      const R a = c, b = T[k];                                 \
      T[k] = (EXPR);                                           \
    }                                                          \
    break;                                                     \
  }

// symbreg_numpy.py:28-36: numpy.divide, then inf and nan become 1.
template <typename R>
__device__ __forceinline__ R np_pdiv(R l, R r) {
  const R q = l / r;
  return __builtin_isfinite(q) ? q : R(1);
}

// sin/cos of the fp32 mode (the asm core gen_asm32.py runs these
// operations in this order): x = k*pi/2 + r, k = rint(x*2/pi), r by a
// three-part Cody-Waite reduction with FMA (|x| < 2^30), cephes sinf/cosf
// polynomials on [-pi/4, pi/4], selected and signed by the quadrant k mod 4.
// About 1 ulp (fp32) below 2^20, 2 up to 2^30; beyond, and for inf/nan, the
// platform libm (nan for inf, as the core's polynomial path gives).
HD float gp_trig32(float x, bool cosine) {
  using namespace asmcore32;
  if (!(__builtin_fabsf(x) < 0x1p30f)) return cosine ? ::cosf(x) : ::sinf(x);
  const float kf = __builtin_rintf(x * kConst[0]);
  float r = __builtin_fmaf(-kf, kConst[1], x);
  r = __builtin_fmaf(-kf, kConst[2], r);
  r = __builtin_fmaf(-kf, kConst[3], r);
  const int q = (int)kf + (cosine ? 1 : 0);
  const float z = r * r;
  float ps = __builtin_fmaf(z, kConst[6], kConst[5]);
  ps = __builtin_fmaf(ps, z, kConst[4]);
  const float s = __builtin_fmaf(r * z, ps, r);
  float pc = __builtin_fmaf(z, kConst[9], kConst[8]);
  pc = __builtin_fmaf(pc, z, kConst[7]);
  const float c = __builtin_fmaf(z * z, pc, __builtin_fmaf(z, -0.5f, 1.0f));
  const float res = (q & 1) ? c : s;
  uint32_t bits;
  memcpy(&bits, &res, 4);
  bits ^= ((uint32_t)q << 30) & 0x80000000u;
  float out;
  memcpy(&out, &bits, 4);
  return out;
}

// sin/cos of the interpreters: fp64 = gp_trig (near-correctly rounded; the
// reference's glibc to the last bit except where glibc misrounds), or with
// EXACT (the redo pass of f_eval_asm) glibc_trig, the reference's libm
// itself; fp32 = gp_trig32.
// gtab: the LDS copy of glibc's two tables (kGlibcLdsDoubles) in EXACT
// kernels.
constexpr int kGlibcLdsDoubles = 440 + 75;
template <bool EXACT>
__device__ __forceinline__ double trig_x(double x, bool cosine, const double* gtab) {
  // (no LDS copy: the tables in global memory)
  return !EXACT ? gp_trig(x, cosine)
         : gtab ? glibc_trig_t(x, cosine, gtab, gtab + 440)
                : glibc_trig(x, cosine);
}
template <bool EXACT>
__device__ __forceinline__ float trig_x(float x, bool cosine, const double*) {
  return gp_trig32(x, cosine);
}

// Interpret one F program over the lane's K cases; T receives the value and
// vbits bit k is set if math.sin/cos saw +-inf for case k (ValueError).
template <int K, typename R, bool EXACT = false>
__device__ __forceinline__ void f_run(const ProgWords& W, const R* xs,
                                      R* stk, int lane, R (&T)[K],
                                      uint32_t& vbits,
                                      const double* gtab = nullptr) {
  constexpr R zero = R(0), one = R(1);
  R o[K];
  FOR_K T[k] = zero;
  uint32_t i = 0;
  for (;;) {
    const uint32_t w = W[i++];
    const uint32_t op = w & 0xffu;
    const uint32_t d = (w >> 8) & 0xffu;
    const uint32_t x = w >> 16;
    if (op == OP_END) break;
    switch (op) {
      case OP_LDV:
        ld_tile<K>(xs, x, lane, T);
        break;
      case OP_LDC: {
        const R c = (R)dbits(W[i], W[i + 1]);
        i += 2;
        FOR_K T[k] = c;
        break;
      }
      case OP_PUSH:
        st_tile<K>(stk, d, lane, T);
        break;
      case OP_PUSHV:
        st_tile<K>(stk, d, lane, T);
        ld_tile<K>(xs, x, lane, T);
        break;
      case OP_PUSHC: {
        st_tile<K>(stk, d, lane, T);
        const R c = (R)dbits(W[i], W[i + 1]);
        i += 2;
        FOR_K T[k] = c;
        break;
      }
      F_BIN(OP_ADD, a + b)
      F_BIN(OP_SUB, a - b)
      F_BIN(OP_RSUB, b - a)
      F_BIN(OP_MUL, a * b)
      F_BIN(OP_DIV, (b == zero) ? one : a / b)    // protectedDiv(a, b)
      F_BIN(OP_RDIV, (a == zero) ? one : b / a)   // protectedDiv(b, a)
      F_BIN(OP_LT, (a < b) ? one : zero)
      F_BIN(OP_GT, (b < a) ? one : zero)
      F_BIN(OP_EQ, (a == b) ? one : zero)
      F_BIN(OP_AND, (a != zero && b != zero) ? one : zero)
      F_BIN(OP_OR, (a != zero || b != zero) ? one : zero)
      F_BIN(OP_NPDIV, np_pdiv(a, b))              // numpy protectedDiv(a, b)
      F_BIN(OP_RNPDIV, np_pdiv(b, a))
      case OP_NEG:
        FOR_K T[k] = -T[k];
        break;
      case OP_SIN:
      case OP_COS:
        FOR_K vbits |= (uint32_t)__builtin_isinf(T[k]) << k;
        if constexpr (EXACT && std::is_same<R, double>::value) {
          if (gtab)
            glibc_trig_k<K>(T, op == OP_COS, gtab, gtab + 440);
          else
            glibc_trig_k<K>(T, op == OP_COS, asmcore::kGlibcSincostab,
                            asmcore::kGlibcToverp);
        } else {
          FOR_K T[k] = trig_x<EXACT>(T[k], op == OP_COS, gtab);
        }
        break;
      case OP_NOT:
        FOR_K T[k] = (T[k] == zero) ? one : zero;
        break;
      case OP_ITE: {
        R c[K];
        ld_tile<K>(stk, d, lane, c);
        ld_tile<K>(stk, d + 1, lane, o);
        FOR_K T[k] = (c[k] != zero) ? o[k] : T[k];
        break;
      }
      default:  // rejected by validate_program(); unreachable
        return;
    }
  }
}

// Stage tile `t` of (X, terms) into LDS as [var][k][lane] doubles.
template <int K, typename R>
__device__ __forceinline__ void f_stage(const Task& a, R* xs,
                                        int64_t t, int stride = kBlock) {
  const int per = K * 64;
  const int total = (a.nv + a.nt) * per;
  const int64_t base = t * per;
  const double* X = (const double*)a.X;
  const double* Tm = (const double*)a.terms;
  for (int i = threadIdx.x; i < total; i += stride) {
    const int v = i / per;
    const int r = i - v * per;
    const int64_t c = base + r;
    double val = 0.0;
    if (c < a.n_cases)
      val = (v < a.nv) ? X[(int64_t)v * a.n_cases + c]
                       : Tm[(int64_t)(v - a.nv) * a.n_cases + c];
    xs[i] = (R)val;
  }
}

// R = double: the fp64 machine (reference parity).  R = float: the fp32
// mode — cases, targets, the tree and d*d in fp32, the sum still in fp64
// double-double.
template <int K, int D, int MODE, typename R, bool EXACT = false>
__global__ __launch_bounds__(kFMaxBlock) void f_eval(Task a) {
  extern __shared__ double lds_d[];
  R* lds = (R*)lds_d;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  R* xs = lds;                                        // [nv][K][64]
  const R* ts = xs + a.nv * K * 64;                   // [nt][K][64]
  // (the stack holds the launch's deepest program, not D: a smaller LDS
  // footprint admits more blocks per CU)
  R* stk = lds + (a.nv + a.nt) * K * 64 + wave * a.sdepth * K * 64;

  const int nwaves = (int)(blockDim.x >> 6);
  // EXACT: glibc's tables after the stacks (launch_f sized the LDS for them)
  const double* gtab = nullptr;
  if (EXACT && a.gtab_lds) {
    double* g = (double*)(lds + (a.nv + a.nt + nwaves * a.sdepth) * K * 64);
    for (int i = threadIdx.x; i < kGlibcLdsDoubles; i += (int)blockDim.x)
      g[i] = i < 440 ? asmcore::kGlibcSincostab[i] : asmcore::kGlibcToverp[i - 440];
    gtab = g;
  }
  const int64_t wave_id = (int64_t)blockIdx.y * nwaves + wave;
  const int64_t slot0 = wave_id * a.P;
  int my_prog = -1;
  if (lane < a.P && slot0 + lane < a.n_slots) my_prog = a.slot_prog[slot0 + lane];
  // lane j < P also holds program j's first word offset (v_readlane below)
  int64_t my_off = my_prog >= 0 ? a.off[my_prog] : 0;
  auto off_of = [&](int j) -> int64_t {
    return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(my_off >> 32), j)
                      << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)my_off, j));
  };
  const int n_mine = [&] {
    int n = 0;
    for (int j = 0; j < a.P; ++j)
      if (__builtin_amdgcn_readlane(my_prog, j) >= 0) n = j + 1;
    return n;
  }();

  double acc_hi = 0.0, acc_lo = 0.0;
  unsigned long long acc_err = ~0ull;
  uint32_t acc_flag = 0;

  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_group;
  const int64_t t1 = min(a.n_tiles, t0 + a.tiles_per_group);
  for (int64_t t = t0; t < t1; ++t) {
    __syncthreads();
    f_stage<K>(a, lds, t, (int)blockDim.x);
    __syncthreads();
    const int64_t case0 = t * (K * 64) + lane;
    // each program's first 64 words: loaded one program ahead, so the load
    // latency hides behind the previous program (tiny programs: it was most
    // of the time)
    uint32_t win = n_mine ? a.code[off_of(0) + lane] : 0u;
    for (int j = 0; j < n_mine; ++j) {
      const int prog = __builtin_amdgcn_readlane(my_prog, j);
      R T[K];
      uint32_t vbits = 0;
      const int64_t off = off_of(j);
      const ProgWords W(a.code + off, win);
      if (j + 1 < n_mine) win = a.code[off_of(j + 1) + lane];
      f_run<K, R, EXACT>(W, xs, stk, lane, T, vbits, gtab);

      double hi = 0.0, lo = 0.0;
      uint32_t hits = 0;                  // HITS_BOOL: wave total (uniform)
      unsigned long long err = ~0ull;
      uint32_t flag = 0;
      FOR_K {
        const int64_t c = case0 + k * 64;
        if (c < a.n_cases) {
          if (MODE == GPE_MODE_MSE) {
            R dlt = T[k];
            for (int q = 0; q < a.nt; ++q) dlt = dlt - ts[(q * K + k) * 64 + lane];
            const R sq_r = dlt * dlt;
            const double sq = (double)sq_r;
            const bool fin = __builtin_isfinite(dlt);
            if (!fin) flag |= GPE_FLAG_NONFINITE_TERM;
            if (sq != sq) flag |= GPE_FLAG_NAN_TERM;
            if (__builtin_isinf(sq)) flag |= GPE_FLAG_INF_TERM;
            uint32_t type = ((vbits >> k) & 1u) ? GPE_ERR_VALUE
                            : (fin && __builtin_isinf(sq)) ? GPE_ERR_OVERFLOW
                                                          : 0u;
            if (type) err = min(err, ((unsigned long long)c << 2) | type);
            double s, e;
            two_sum(hi, sq, s, e);
            hi = s;
            lo = lo + e;
            if (a.case_out) a.case_out[(size_t)prog * a.n_cases + c] = sq;
          } else if (a.case_out) {
            const bool pred = T[k] != R(0);
            const bool lab = ts[k * 64 + lane] != R(0);
            a.case_out[(size_t)prog * a.n_cases + c] = (pred == lab) ? 1.0 : 0.0;
          }
        }
        if (MODE != GPE_MODE_MSE) {       // count matches with one ballot
          const bool match = c < a.n_cases &&
                             ((T[k] != R(0)) == (ts[k * 64 + lane] != R(0)));
          hits += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(match));
        }
      }
      if (MODE == GPE_MODE_MSE) {
        // wave reduction (fixed butterfly order)
        for (int m = 32; m >= 1; m >>= 1) {
          const double ohi = shfl_xor_d(hi, m);
          const double olo = shfl_xor_d(lo, m);
          dd_add(hi, lo, ohi, olo);
        }
        uint32_t f = flag;
        for (int m = 32; m >= 1; m >>= 1) f |= __shfl_xor(f, m, 64);
        if (__builtin_amdgcn_ballot_w64(err != ~0ull)) {
          for (int m = 32; m >= 1; m >>= 1) {
            const unsigned long long oe = __shfl_xor(err, m, 64);
            err = min(err, oe);
          }
        }
        if (lane == j) {
          dd_add(acc_hi, acc_lo, hi, lo);
          acc_err = min(acc_err, err);
          acc_flag |= f;
        }
      } else if (lane == j) {
        acc_hi += (double)hits;
      }
    }
  }
  if (my_prog >= 0) {
    double* p = a.part + ((size_t)blockIdx.x * a.n_slots + slot0 + lane) * 2;
    p[0] = acc_hi;
    p[1] = acc_lo;
    if (MODE == GPE_MODE_MSE) {
      if (acc_err != ~0ull) atomicMin(&a.first_err[my_prog], acc_err);
      if (acc_flag) atomicOr(&a.flags[my_prog], acc_flag);
    }
  }
}

// ---------------------------------------------------------------- B ----
__device__ __forceinline__ void b_run(const uint32_t* pc, const uint32_t* xs,
                                      uint32_t* stk, int lane, uint32_t& T) {
  T = 0;
  const ProgWords W(pc, lane);
  uint32_t i = 0;
  for (;;) {
    const uint32_t w = W[i++];
    const uint32_t op = w & 0xffu;
    const uint32_t d = (w >> 8) & 0xffu;
    const uint32_t x = w >> 16;
    if (op == OP_END) break;
    const uint32_t cmask = x ? 0xffffffffu : 0u;
    switch (op) {
      case OP_LDV: T = xs[x * 64 + lane]; break;
      case OP_LDC: T = cmask; break;
      case OP_PUSH: stk[d * 64 + lane] = T; break;
      case OP_PUSHV: stk[d * 64 + lane] = T; T = xs[x * 64 + lane]; break;
      case OP_PUSHC: stk[d * 64 + lane] = T; T = cmask; break;
      case OP_AND + 0: T = stk[d * 64 + lane] & T; break;
      case OP_AND + 1: T = xs[x * 64 + lane] & T; break;
      case OP_AND + 2: T = cmask & T; break;
      case OP_OR + 0: T = stk[d * 64 + lane] | T; break;
      case OP_OR + 1: T = xs[x * 64 + lane] | T; break;
      case OP_OR + 2: T = cmask | T; break;
      case OP_XOR + 0: T = stk[d * 64 + lane] ^ T; break;
      case OP_XOR + 1: T = xs[x * 64 + lane] ^ T; break;
      case OP_XOR + 2: T = cmask ^ T; break;
      case OP_NOT: T = ~T; break;
      case OP_ITE: {
        const uint32_t c = stk[d * 64 + lane];
        const uint32_t v = stk[(d + 1) * 64 + lane];
        T = (c & v) | (~c & T);
        break;
      }
      default:  // rejected by validate_program(); unreachable
        return;
    }
  }
}

template <int D>
__global__ __launch_bounds__(kBlock) void b_eval(Task a) {
  extern __shared__ uint32_t ldsw[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  uint32_t* xs = ldsw;                       // [nv][64]
  const uint32_t* outp = xs + a.nv * 64;     // [64]
  uint32_t* stk = ldsw + (a.nv + 1) * 64 + wave * D * 64;

  const int64_t wave_id = (int64_t)blockIdx.y * kWaves + wave;
  const int64_t slot0 = wave_id * a.P;
  int my_prog = -1;
  if (lane < a.P && slot0 + lane < a.n_slots) my_prog = a.slot_prog[slot0 + lane];
  // lane j < P also holds program j's first word offset (v_readlane below)
  int64_t my_off = my_prog >= 0 ? a.off[my_prog] : 0;
  double acc = 0.0;
  const uint32_t* X = (const uint32_t*)a.X;
  const uint32_t* O = (const uint32_t*)a.terms;

  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_group;
  const int64_t t1 = min(a.n_tiles, t0 + a.tiles_per_group);
  for (int64_t t = t0; t < t1; ++t) {
    __syncthreads();
    for (int i = threadIdx.x; i < (a.nv + 1) * 64; i += kBlock) {
      const int v = i >> 6;
      const int64_t wd = t * 64 + (i & 63);
      uint32_t val = 0;
      if (wd < a.n_units) val = (v < a.nv) ? X[(int64_t)v * a.n_units + wd] : O[wd];
      xs[i] = val;
    }
    __syncthreads();
    const int64_t wd = t * 64 + lane;
    uint32_t vmask = 0;
    if (wd < a.n_units) {
      const int64_t rem = a.n_cases - wd * 32;
      vmask = rem >= 32 ? 0xffffffffu : ((1u << rem) - 1u);
    }
    for (int j = 0; j < a.P; ++j) {
      const int prog = __builtin_amdgcn_readlane(my_prog, j);
      if (prog < 0) break;
      uint32_t T;
      const int64_t off = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                              (int)(my_off >> 32), j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)my_off, j));
      b_run(a.code + off, xs, stk, lane, T);
      uint32_t h = (uint32_t)__builtin_popcount(~(T ^ outp[lane]) & vmask);
      for (int m = 32; m >= 1; m >>= 1) h += __shfl_xor(h, m, 64);
      if (lane == j) acc += (double)h;
    }
  }
  if (my_prog >= 0) {
    double* p = a.part + ((size_t)blockIdx.x * a.n_slots + slot0 + lane) * 2;
    p[0] = acc;
    p[1] = 0.0;
  }
}

// Tiny case sets (n_units <= 16 words, e.g. parity-6's 64 cases = 2 words):
// b_eval would leave 62 of 64 lanes idle, so here each lane interprets its
// own program — G lanes (G = n_units rounded up to a power of two) share a
// program, one 32-case word each, and a wave runs 64/G programs (the plan's
// P) side by side.  Per-lane program counters; the op switch diverges
// across the wave's programs (they are cost-sorted, so their lengths are
// close); the words are the same b_run executes.
template <int D>
__global__ __launch_bounds__(kBlock) void b_eval_lanes(Task a, int G) {
  extern __shared__ uint32_t ldsw[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  uint32_t* xs = ldsw;                       // [nv][64], then the outputs
  const uint32_t* outp = xs + a.nv * 64;
  uint32_t* stk = ldsw + (a.nv + 1) * 64 + wave * D * 64;
  const uint32_t* X = (const uint32_t*)a.X;
  const uint32_t* O = (const uint32_t*)a.terms;
  for (int i = threadIdx.x; i < (a.nv + 1) * 64; i += kBlock) {
    const int v = i >> 6;
    const int64_t wd = i & 63;
    uint32_t val = 0;
    if (wd < a.n_units) val = (v < a.nv) ? X[(int64_t)v * a.n_units + wd] : O[wd];
    xs[i] = val;
  }
  __syncthreads();
  const int64_t wave_id = (int64_t)blockIdx.y * kWaves + wave;
  const int64_t slot = wave_id * a.P + lane / G;
  const int wd = lane & (G - 1);
  const int prog = slot < a.n_slots ? a.slot_prog[slot] : -1;
  bool active = prog >= 0;
  const uint32_t* pc = a.code + (active ? a.off[prog] : 0);
  uint32_t T = 0;
  uint32_t w = active ? pc[0] : (uint32_t)OP_END;
  while (__builtin_amdgcn_ballot_w64(active)) {
    if (active) {
      const uint32_t op = w & 0xffu;
      const uint32_t d = (w >> 8) & 0xffu;
      const uint32_t x = w >> 16;
      if (op == OP_END) {
        active = false;
      } else {
        w = *++pc;                           // next word, ahead of its use
        const uint32_t cmask = x ? 0xffffffffu : 0u;
        switch (op) {
          case OP_LDV: T = xs[x * 64 + wd]; break;
          case OP_LDC: T = cmask; break;
          case OP_PUSH: stk[d * 64 + lane] = T; break;
          case OP_PUSHV: stk[d * 64 + lane] = T; T = xs[x * 64 + wd]; break;
          case OP_PUSHC: stk[d * 64 + lane] = T; T = cmask; break;
          case OP_AND + 0: T = stk[d * 64 + lane] & T; break;
          case OP_AND + 1: T = xs[x * 64 + wd] & T; break;
          case OP_AND + 2: T = cmask & T; break;
          case OP_OR + 0: T = stk[d * 64 + lane] | T; break;
          case OP_OR + 1: T = xs[x * 64 + wd] | T; break;
          case OP_OR + 2: T = cmask | T; break;
          case OP_XOR + 0: T = stk[d * 64 + lane] ^ T; break;
          case OP_XOR + 1: T = xs[x * 64 + wd] ^ T; break;
          case OP_XOR + 2: T = cmask ^ T; break;
          case OP_NOT: T = ~T; break;
          case OP_ITE: {
            const uint32_t c = stk[d * 64 + lane];
            const uint32_t v = stk[(d + 1) * 64 + lane];
            T = (c & v) | (~c & T);
            break;
          }
          default:  // rejected by validate_program(); unreachable
            active = false;
            break;
        }
      }
    }
  }
  uint32_t vmask = 0;
  if (wd < a.n_units) {
    const int64_t rem = a.n_cases - (int64_t)wd * 32;
    vmask = rem >= 32 ? 0xffffffffu : ((1u << rem) - 1u);
  }
  uint32_t h = (uint32_t)__builtin_popcount(~(T ^ outp[wd]) & vmask);
  for (int m = G >> 1; m >= 1; m >>= 1) h += __shfl_xor(h, m, 64);
  if (wd == 0 && prog >= 0) {
    double* p = a.part + (size_t)slot * 2;   // one tile group
    p[0] = (double)h;
    p[1] = 0.0;
  }
}

// Sum partials over tile groups (fixed order) and scatter to program order.
__global__ __launch_bounds__(256) void reduce_groups(
    const double* part, int64_t n_slots, int n_groups,
    const int32_t* slot_prog, double* out_hi, double* out_lo) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slots) return;
  const int prog = slot_prog[s];
  if (prog < 0) return;
  double hi = 0.0, lo = 0.0;
  for (int g = 0; g < n_groups; ++g) {
    const double* p = part + ((size_t)g * n_slots + s) * 2;
    dd_add(hi, lo, p[0], p[1]);
  }
  out_hi[prog] = hi;
  out_lo[prog] = lo;
}

// Diagnostic: the device's elementary functions on host-given inputs.
__global__ void math_probe(int fn, const double* x, double* y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  double sn, cs;
  gp_sincos(v, sn, cs);
  y[i] = fn == 0 ? sn : fn == 1 ? cs : fn == 2 ? v * v : fn == 3 ? sin(v)
       : fn == 4 ? cos(v) : fn >= 11 ? glibc_trig(v, fn == 12)
       : (double)gp_trig32((float)v, fn == 10);
}

}  // namespace
