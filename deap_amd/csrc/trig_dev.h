// Part of gpeval.hip's single translation unit (included there once, in
// order, inside the library's anonymous namespace for device code): sin/cos: the table-driven near-correctly-rounded
// pair and the restatement of glibc 2.35's __sin/__cos/__branred.
#pragma once
namespace {

// ------------------------------------------------------ sin/cos ----------
// Near-correctly-rounded sin/cos.  The reference evaluates math.sin/cos
// (glibc 2.35, misrounded in ~0.1-0.2 % of calls); ocml's f64 sin/cos are
// off by one ulp in ~3.5 % of calls, which ill-conditioned GP trees amplify
// past the 1e-12 SSE tolerance.  This one misrounded none of 2.4 million
// random arguments, so device and reference differ only
// where glibc misrounds.
//
// Table-driven on a grid of step c = pi/256 (gen_trig_table.py):
// k = rint(x/c) from one fma with 1.5*2^52 (its low word is k), j = k mod
// 512, x = k*c + r with |r| <= pi/512, r = t + rl:
//   |x| < 2^14 (FAST): t = x - k*S1 exactly (one fma: S1 = c rounded, and
//     x - k*S1, a multiple of 2^-60 below 2^-7, fits 53 bits), rl = k*(-S2)
//     (|k| < 2^21, |rl| < 2^-40, error < 2^-92)
//   2^14 <= |x| < 2^40: error-free product k*C1, two TwoSums over
//     k*(C1 + C2 + C3), |error| < 2^-110
// With S = sin(j c) = Sh + Sl and C = cos(j c) = Ch + Cl (double-doubles,
// table entries j and j + 128), z = (t + rl)^2:
//   a  = Sh + Ch*t                                   (one fma, error ae exact)
//   sin(x) = a + [Sl + Cl*t + Ch*rl + ae + z*(Sh*Pc(z) + Ch*(t+rl)*Ps(z))]
// where Pc(z) = (cos r - 1)/z and Ps(z) = (sin r - r)/(r z): the bracket is
// below 2^-15 of the result, so its rounding errors stay ~2^-68 of it.
// 21 fp64 operations below 2^14.  cos(x) = sin(x + pi/2): entries j + 128
// and j + 256.  |x| >= 2^40 (and inf/nan): glibc_trig, the reference's own
// libm bit for bit.
#define HD __host__ __device__ __forceinline__
HD void fast_two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  e = b - (s - a);
}
HD void two_sum_h(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}
// ------------------------------------------- the reference's libm ----
// Attribution: this section (namespace glibc: the constants, taylor_sin,
// reduce_sincos, branred_half / branred, do_sin / do_cos, glibc_trig_t) and
// the tables it reads restate algorithms of the GNU C Library 2.35,
// sysdeps/ieee754/dbl-64/s_sin.c, branred.c, sincostab.c and usncs.h / branred.h
// (Copyright (C) 2001-2022 Free Software Foundation, Inc.; IBM Accurate
// Mathematical Library), which glibc distributes under the GNU Lesser
// General Public License, version 2.1 or later.  The same algorithms are
// emitted as gfx950 assembly by gen_asm.py (glibc_seq3 / glibc_seq4,
// branred_ops).
// glibc_sin / glibc_cos: glibc 2.35's sin/cos (sysdeps/ieee754/dbl-64/
// s_sin.c __sin/__cos, do_sin, do_cos, reduce_sincos, TAYLOR_SIN; branred.c
// __branred for |x| >= 105414350), restated operation for operation with the
// fused multiply-adds the x86-64 FMA build of s_sin.c contains (gcc's
// contraction of the C source; branred.c is built without contraction), so
// that they return the host libm's — the reference's math.sin/cos — bits:
// tests/test_lib.py checks the host-compiled twin against the host's libm on
// millions of arguments over the whole double range.  Tables: glibc's
// __sincostab (sin/cos(i/128) as double-doubles) and toverp (2/pi in base
// 2^24), regenerated from their definitions by gen_trig_table.py.
// Branchy (per-lane paths by |x| range): used where exactness matters more
// than speed — gp_trig beyond 2^40 and the redo pass of ill-conditioned
// (program, tile) pairs.
namespace glibc {
HD uint32_t hi_word(double x) {
  uint64_t b;
  memcpy(&b, &x, 8);
  return (uint32_t)(b >> 32);
}
HD uint32_t lo_word(double x) {
  uint64_t b;
  memcpy(&b, &x, 8);
  return (uint32_t)b;
}
HD double from_words(uint32_t h, uint32_t l) {
  const uint64_t b = ((uint64_t)h << 32) | l;
  double x;
  memcpy(&x, &b, 8);
  return x;
}
constexpr double SN3 = -1.66666666666664880952546298448555E-01,
                 SN5 = 8.33333214285722277379541354343671E-03,
                 CS2 = 4.99999999999999999999950396842453E-01,
                 CS4 = -4.16666666666664434524222570944589E-02,
                 CS6 = 1.38888874007937613028114285595617E-03,
                 S1 = -0x1.5555555555555p-3, S2 = 0x1.1111111110ECEp-7,
                 S3 = -0x1.a01a019db08b8p-13, S4 = 0x1.71de27b9a7ed9p-19,
                 S5 = -0x1.addffc2fcdf59p-26, BIG = 0x1.8p45,
                 HP0 = 0x1.921FB54442D18p0, HP1 = 0x1.1A62633145C07p-54,
                 MP1 = 0x1.921FB58000000p0, MP2 = -0x1.DDE973C000000p-27,
                 PP3 = -0x1.CB3B398000000p-55, PP4 = -0x1.d747f23e32ed7p-83,
                 HPINV = 0x1.45F306DC9C883p-1, TOINT = 0x1.8p52,
                 // branred.h: hp0 split by Veltkamp (mp1 + mp2 == hp0)
                 BMP2 = -0x1.dde9740000000p-27, SPLIT = 134217729.0,
                 BBIG = 0x1.8p52, BBIG1 = 0x1.8p54, TM600 = 0x1p-600,
                 TM24 = 0x1p-24, T576 = 0x1p576;
#define GFMA __builtin_fma
HD double taylor_sin(double xx, double a, double da) {
  double p = GFMA(xx, S5, S4);
  p = GFMA(p, xx, S3);
  p = GFMA(p, xx, S2);
  p = GFMA(p, xx, S1);
  const double h = da * 0.5;
  const double q = GFMA(p, a, -h);
  return a + GFMA(q, xx, da);
}
HD int reduce_sincos(double x, double& a, double& da) {
  const double t = GFMA(x, HPINV, TOINT);
  const double xn = t - TOINT;
  const double y = GFMA(xn, -MP2, GFMA(-xn, MP1, x));
  const int n = (int)(lo_word(t) & 3u);
  const double t2 = GFMA(-xn, PP3, y);
  const double db = GFMA(-xn, PP3, y - t2);
  const double b = GFMA(-xn, PP4, t2);
  a = b;
  da = GFMA(-xn, PP4, t2 - b) + db;
  return n;
}
// branred.c: x * 2/pi to ~136 bits from the 24-bit digits of 2/pi, x split
// in two 26-bit halves; returns the quadrant and a + aa in [-pi/4, pi/4]
HD double branred_half(double xh, double& sum, double& bb_out,
                        const double* kGlibcToverp) {
  double r[6], s, t, bb;
  int k = (int)((hi_word(xh) >> 20) & 2047);
  k = (k - 450) / 24;
  if (k < 0) k = 0;
  double gor = from_words(hi_word(T576) - (uint32_t)((k * 24) << 20), lo_word(T576));
  for (int i = 0; i < 6; ++i) {
    r[i] = xh * kGlibcToverp[k + i] * gor;
    gor *= TM24;
  }
  sum = 0.0;
  for (int i = 0; i < 3; ++i) {
    s = (r[i] + BBIG) - BBIG;
    sum += s;
    r[i] -= s;
  }
  t = 0.0;
  for (int i = 0; i < 6; ++i) t += r[5 - i];
  bb = (((((r[0] - t) + r[1]) + r[2]) + r[3]) + r[4]) + r[5];
  s = (t + BBIG) - BBIG;
  sum += s;
  t -= s;
  const double b = t + bb;
  bb_out = (t - b) + bb;
  s = (sum + BBIG1) - BBIG1;
  sum -= s;
  return b;
}
HD int branred(double x, double& a, double& aa, const double* toverp) {
  x *= TM600;
  double t = x * SPLIT;
  const double x1 = t - (t - x);
  const double x2 = x - x1;
  double sum1, sum2, bb1, bb2;
  const double b1 = branred_half(x1, sum1, bb1, toverp);
  const double b2 = branred_half(x2, sum2, bb2, toverp);
  double sum = sum1 + sum2;
  double b = b1 + b2;
  double bb = (__builtin_fabs(b1) > __builtin_fabs(b2)) ? (b1 - b) + b2 : (b2 - b) + b1;
  if (b > 0.5) {
    b -= 1.0;
    sum += 1.0;
  } else if (b < -0.5) {
    b += 1.0;
    sum -= 1.0;
  }
  double s = b + (bb + bb1 + bb2);
  t = ((b - s) + bb) + (bb1 + bb2);
  b = s * SPLIT;
  const double t1 = b - (b - s);
  const double t2 = s - t1;
  b = s * HP0;
  bb = (((t1 * MP1 - b) + t1 * BMP2) + t2 * MP1) + (t2 * BMP2 + s * HP1 + t * HP0);
  s = b + bb;
  t = (b - s) + bb;
  a = s;
  aa = t;
  return ((int)sum) & 3;
}
// do_sin (n even) / do_cos (n odd) of s_sin.c as ONE instruction stream
// (then negated if n & 2, as do_sincos does): the two bodies differ only in
// where dx enters and in which table words play which part, so a wave whose
// lanes take different paths runs one body with per-lane selects instead of
// both bodies one after the other.  Operation for operation the same
// roundings as glibc (do_cos's fma(-s, ssn, ccs) is fma(s, -ssn, ccs), ...).
// `tab`: __sincostab (global memory, or an LDS copy).
HD double do_sincos(double a, double da, int n, const double* tab) {
  const bool isc = (n & 1) != 0;
  const double ax = __builtin_fabs(a);
  // do_sin: if (x <= 0) dx = -dx; do_cos: if (x < 0) dx = -dx
  const double dxs = (isc ? a < 0.0 : a <= 0.0) ? -da : da;
  const double u = ax + BIG;
  const double xr = ax - (u - BIG);
  const double v = isc ? xr + dxs : xr;               // do_cos folds dx in
  const double xx = v * v;
  const double m = v * xx;
  const double p = GFMA(xx, SN5, SN3);
  const double t = GFMA(m, p, isc ? v : dxs);
  const double s = isc ? t : t + xr;
  const double w = GFMA(GFMA(xx, CS6, CS4), xx, CS2) * xx;
  const double c = GFMA(isc ? 0.0 : dxs, xr, w);      // do_cos: c = w
  const int k = (int)(lo_word(u) << 2);
  // sin: (A, Aa, B, Bb) = (sn, ssn, cs, ccs); cos: (cs, ccs, -sn, -ssn)
  const int ka = isc ? k + 2 : k, kb = isc ? k : k + 2;
  const double A = tab[ka], Aa = tab[ka + 1];
  double B = tab[kb], Bb = tab[kb + 1];
  if (isc) {
    B = -B;
    Bb = -Bb;
  }
  double cor = GFMA(s, Bb, Aa);
  cor = GFMA(-c, A, cor);
  cor = GFMA(s, B, cor);
  double r = A + cor;
  if (!isc) r = __builtin_copysign(r, a);
  if (!isc && ax < 0.126) r = taylor_sin(a * a, a, da);
  return (n & 2) ? -r : r;
}
#undef GFMA
}  // namespace glibc

// glibc 2.35 __sin / __cos: the argument ranges of s_sin.c reduce to one
// (a, da, n) per lane, then one do_sincos (above); __branred only where a
// lane needs it.  `tab`/`toverp`: the two tables (global or LDS copies).
HD double glibc_trig_t(double x, bool cosine, const double* tab,
                       const double* toverp) {
  using namespace glibc;
  const uint32_t k = 0x7fffffffu & hi_word(x);
  double a = x, da = 0.0;
  int n = cosine ? 1 : 0;                     // |x| < 0.855469: do_sin/do_cos(x, 0)
  if (k >= 0x3feb6000u && k < 0x400368fdu) {  // |x| < 2.426265
    const double y = HP0 - __builtin_fabs(x);
    if (cosine) {                             // do_sin(y + hp1, ...)
      a = y + HP1;
      da = (y - a) + HP1;
      n = 0;
    } else {                                  // copysign(do_cos(y, hp1), x)
      a = y;
      da = HP1;
      n = x < 0.0 ? 3 : 1;                    // (do_cos is positive here)
    }
  } else if (k >= 0x400368fdu && k < 0x419921FBu) {   // |x| < 105414350
    n = reduce_sincos(x, a, da) + (cosine ? 1 : 0);
  } else if (k >= 0x419921FBu && k < 0x7ff00000u) {
    n = branred(x, a, da, toverp) + (cosine ? 1 : 0);
  }
  const double r = do_sincos(a, da, n, tab);
  if (k >= 0x7ff00000u) return x / x;         // nan: inf or nan
  if (cosine ? k < 0x3e400000u : k < 0x3e500000u) return cosine ? 1.0 : x;
  return r;
}
HD double glibc_trig(double x, bool cosine) {
  return glibc_trig_t(x, cosine, asmcore::kGlibcSincostab, asmcore::kGlibcToverp);
}
// glibc_trig_t over the K cases of a lane at once (the exact interpreter):
// one range test, one reduce_sincos and one do_sincos stream shared by the
// K chains, so a wave's branches are taken once per node, not once per case.
template <int K>
HD void glibc_trig_k(double (&x)[K], bool cosine, const double* tab,
                     const double* toverp) {
  using namespace glibc;
  uint32_t kw[K];
  double a[K], da[K];
  int n[K];
  bool any_red = false, any_big = false;
  for (int k = 0; k < K; ++k) {
    kw[k] = 0x7fffffffu & hi_word(x[k]);
    const double y = HP0 - __builtin_fabs(x[k]);
    const double ac = y + HP1;
    const bool mid = kw[k] >= 0x3feb6000u && kw[k] < 0x400368fdu;  // < 2.426265
    a[k] = mid ? (cosine ? ac : y) : x[k];
    da[k] = mid ? (cosine ? (y - ac) + HP1 : HP1) : 0.0;
    n[k] = mid ? (cosine ? 0 : (x[k] < 0.0 ? 3 : 1)) : (cosine ? 1 : 0);
    any_red |= kw[k] >= 0x400368fdu && kw[k] < 0x419921FBu;
    any_big |= kw[k] >= 0x419921FBu && kw[k] < 0x7ff00000u;
  }
  if (any_red) {
    for (int k = 0; k < K; ++k) {
      double ar, dar;
      const int nr = reduce_sincos(x[k], ar, dar) + (cosine ? 1 : 0);
      if (kw[k] >= 0x400368fdu && kw[k] < 0x419921FBu) {
        a[k] = ar;
        da[k] = dar;
        n[k] = nr;
      }
    }
  }
  if (any_big) {
    for (int k = 0; k < K; ++k)
      if (kw[k] >= 0x419921FBu && kw[k] < 0x7ff00000u)
        n[k] = branred(x[k], a[k], da[k], toverp) + (cosine ? 1 : 0);
  }
  for (int k = 0; k < K; ++k) {
    const double r = do_sincos(a[k], da[k], n[k], tab);
    x[k] = kw[k] >= 0x7ff00000u ? x[k] - x[k]       // inf, nan -> nan
           : (cosine ? kw[k] < 0x3e400000u : kw[k] < 0x3e500000u) ? (cosine ? 1.0 : x[k])
           : r;
  }
}
HD double glibc_sin(double x) { return glibc_trig(x, false); }
HD double glibc_cos(double x) { return glibc_trig(x, true); }

HD double gp_trig(double x, bool cosine) {
  using namespace asmcore;
  // kTrigConst: INV, S1, 0, -S2, LIM, TINY, FAST, Ps0 | Ps1, Ps2, Pc1,
  // Pc2, C1, C2, C3, MAGIC (Pc0 = -1/2)
  const double* kc = kTrigConst;
  const double ax = __builtin_fabs(x);
  if (!(ax < kc[4])) return glibc_trig(x, cosine);   // also nan/inf
  if (!cosine && ax < kc[5]) return x;   // correctly rounded, keeps sin(-0)
  // k as the asm cores form it: the low word of kb is k (two's complement)
  const double kb = __builtin_fma(x, kc[0], kc[15]);
  const double kd = kb - kc[15];
  uint64_t kbits;
  memcpy(&kbits, &kb, 8);
  const int j = (int)(kbits & 511u) + (cosine ? 128 : 0);
  double t, rl;
  if (ax < kc[6]) {
    t = __builtin_fma(-kd, kc[1], x);
    rl = kd * kc[3];
  } else {
    const double p1 = kd * kc[12];
    const double p1e = __builtin_fma(kd, kc[12], -p1);
    const double u = x - p1;             // exact (Sterbenz)
    double s, e1, s2, e2;
    two_sum_h(u, -p1e, s, e1);
    const double p2 = kd * kc[13];
    const double p2e = __builtin_fma(kd, kc[13], -p2);
    two_sum_h(s, -p2, s2, e2);
    double rest = e1 + e2;
    rest = rest - p2e;
    rest = __builtin_fma(-kd, kc[14], rest);
    two_sum_h(s2, rest, t, rl);
  }
  const double rr = t + rl;
  const double z = rr * rr;
  const double sh = kTrigTable[2 * j], sl = kTrigTable[2 * j + 1];
  const double ch = kTrigTable[2 * j + 256], cl = kTrigTable[2 * j + 257];
  double ps = __builtin_fma(z, kc[9], kc[8]);
  ps = __builtin_fma(ps, z, kc[7]);
  double pc = __builtin_fma(z, kc[11], kc[10]);
  pc = __builtin_fma(pc, z, -0.5);
  const double a = __builtin_fma(ch, t, sh);
  const double d = sh - a;                 // exact (Sterbenz)
  const double ae = __builtin_fma(ch, t, d);
  const double h = rr * ps;
  const double g = ch * h;
  const double tails = __builtin_fma(sh, pc, g);
  double sm = __builtin_fma(cl, t, sl);
  sm = __builtin_fma(ch, rl, sm);
  sm = sm + ae;
  sm = __builtin_fma(z, tails, sm);
  return a + sm;
}
HD void gp_sincos(double x, double& sn, double& cs) {
  sn = gp_trig(x, false);
  cs = gp_trig(x, true);
}

}  // namespace
