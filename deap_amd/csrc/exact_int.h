// Part of gpeval.hip's single translation unit (included there once, in
// order, inside the library's anonymous namespace for device code): Python's exact ints — the device's 1088-bit
// xint and the host's unbounded hbig.
#pragma once
namespace {

// ------------------------------------------------------------ exact ints --
// The reference evaluates with Python numbers: an int constant (rand101,
// folded subtrees) or protectedDiv's int 1 (examples/gp/symbreg.py:29-33,
// spambase.py:47-49) stays an exact int through operator.add/sub/mul/neg,
// int / int rounds the exact ratio once, int-float comparisons are exact.
// Where a program's ints can pass 2**53 (flatten.py _int_bounds) a float64
// no longer reproduces that, and the exact pass re-evaluates the program
// with this value type: a float, or an int as sign + 1088-bit magnitude.
// Errors as CPython raises them, at the first one in evaluation order:
// float(int) of an int at or past 2**1024 after rounding (a mixed int-float
// operation, sin/cos of an int, the error formula) and int / int past the
// float range are OverflowError; sin/cos(+-inf) ValueError.  An int past the
// 1088 bits this pass holds (the reference keeps going: its ints are
// unbounded) ends the case with E_RANGE: the host evaluates the program
// again with unbounded ints (bigint_host.h, run_exact_host).
namespace xint {
constexpr int kLimbs = 17;               // 1088-bit magnitudes
constexpr int kWords = 2 * kLimbs;       // uint32 words of an int constant
// = GPE_ERR_VALUE / GPE_ERR_OVERFLOW, and E_RANGE for the capacity
enum : uint32_t { E_NONE = 0, E_VALUE = 1, E_OVERFLOW = 2, E_RANGE = 3 };
struct Mag {
  uint64_t w[kLimbs];
};
struct Num {
  bool isint;
  bool neg;          // ints: sign (never set on 0)
  double f;          // floats
  Mag m;             // ints: |value|
};

HD Mag mag_small(uint64_t v) {
  Mag r;
  r.w[0] = v;
  for (int i = 1; i < kLimbs; ++i) r.w[i] = 0;
  return r;
}
HD int used(const Mag& a) {              // limbs up to the highest nonzero one
  for (int i = kLimbs - 1; i >= 0; --i)
    if (a.w[i]) return i + 1;
  return 0;
}
HD bool mag_zero(const Mag& a) { return used(a) == 0; }
HD int mag_cmp(const Mag& a, const Mag& b) {
  for (int i = kLimbs - 1; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
HD Mag mag_add(const Mag& a, const Mag& b, bool& ovf) {
  Mag r;
  uint64_t c = 0;
  for (int i = 0; i < kLimbs; ++i) {
    const uint64_t s = a.w[i] + c;
    const uint64_t c1 = s < c;
    r.w[i] = s + b.w[i];
    c = c1 | (r.w[i] < s);
  }
  ovf |= c != 0;
  return r;
}
HD Mag mag_sub(const Mag& a, const Mag& b) {          // a >= b
  Mag r;
  uint64_t br = 0;
  for (int i = 0; i < kLimbs; ++i) {
    const uint64_t d = a.w[i] - b.w[i];
    const uint64_t b1 = a.w[i] < b.w[i];
    r.w[i] = d - br;
    br = b1 | (d < br);
  }
  return r;
}
HD Mag mag_mul(const Mag& a, const Mag& b, bool& ovf) {
  Mag r = mag_small(0);
  const int la = used(a), lb = used(b);
  if (!la || !lb) return r;
  if (la + lb - 1 > kLimbs) {            // at least 2^(64 (la + lb - 2))
    ovf = true;
    return r;
  }
  uint64_t p[kLimbs + 1];                // la + lb <= kLimbs + 1 limbs
  for (int i = 0; i <= kLimbs; ++i) p[i] = 0;
  for (int i = 0; i < la; ++i) {
    uint64_t carry = 0;
    for (int j = 0; j < lb; ++j) {
      const unsigned __int128 t = (unsigned __int128)a.w[i] * b.w[j] + p[i + j] + carry;
      p[i + j] = (uint64_t)t;
      carry = (uint64_t)(t >> 64);
    }
    p[i + lb] = carry;
  }
  ovf |= p[kLimbs] != 0;
  for (int i = 0; i < kLimbs; ++i) r.w[i] = p[i];
  return r;
}
HD int bits64(uint64_t v) { return v ? 64 - __builtin_clzll(v) : 0; }
template <int N>
HD int bitlen(const uint64_t (&w)[N]) {
  for (int i = N - 1; i >= 0; --i)
    if (w[i]) return 64 * i + bits64(w[i]);
  return 0;
}
template <int N>
HD int bit_at(const uint64_t (&w)[N], int b) {
  return b < 0 || b >= 64 * N ? 0 : (int)((w[b >> 6] >> (b & 63)) & 1u);
}
template <int N>
HD bool any_below(const uint64_t (&w)[N], int b) {     // a bit < b set
  for (int i = 0; i < N && 64 * i < b; ++i) {
    const int k = b - 64 * i;
    const uint64_t mask = k >= 64 ? ~0ull : ((1ull << k) - 1);
    if (w[i] & mask) return true;
  }
  return false;
}
template <int N>
HD uint64_t bits_from(const uint64_t (&w)[N], int b) {  // 64 bits from bit b
  const int i = b >> 6, sh = b & 63;
  uint64_t lo = i < N ? w[i] >> sh : 0;
  if (sh && i + 1 < N) lo |= w[i + 1] << (64 - sh);
  return lo;
}
// round-to-nearest-even of (w + sticky * tiny) * 2^e2 to a double, as
// CPython's float(int) and int / int round: 53 bits, fewer below 2^-1022
// (subnormals, down to zero), ovf when the rounded value reaches 2^1024
template <int N>
HD double round_mag(const uint64_t (&w)[N], bool sticky, int e2, bool& ovf) {
  const int nb = bitlen(w);
  if (nb == 0) return 0.0;
  const int p = nb - 1 + e2;             // the leading bit's exponent
  if (p >= 1024) {
    ovf = true;
    return __builtin_inf();
  }
  const int keep = p >= -1022 ? 53 : p + 1075;          // may be <= 0
  const int sh = nb - keep;              // low bits dropped
  if (sh <= 0) return ldexp((double)w[0], e2);          // exact
  uint64_t mant = keep > 0 ? bits_from(w, sh) & ((1ull << keep) - 1) : 0;
  const int rb = bit_at(w, sh - 1);
  const bool rest = sticky || any_below(w, sh - 1);
  if (rb && (rest || (mant & 1u))) ++mant;              // <= 2^53: exact
  const double v = ldexp((double)mant, sh + e2);
  ovf |= __builtin_isinf(v);
  return v;
}

HD Num from_f(double f) {
  Num r;
  r.isint = false;
  r.neg = false;
  r.f = f;
  r.m = mag_small(0);
  return r;
}
HD Num from_int(bool neg, const Mag& m) {
  Num r;
  r.isint = true;
  r.m = m;
  r.neg = neg && !mag_zero(m);
  r.f = 0.0;
  return r;
}
// kWords-word two's complement, little-endian 32-bit words (flatten.py)
HD Num from_words(const uint32_t* w) {
  Mag m;
  for (int i = 0; i < kLimbs; ++i) m.w[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  const bool neg = (m.w[kLimbs - 1] >> 63) != 0;
  if (neg) {                              // magnitude = ~m + 1
    uint64_t c = 1;
    for (int i = 0; i < kLimbs; ++i) {
      m.w[i] = ~m.w[i] + c;
      c = c && m.w[i] == 0;
    }
  }
  return from_int(neg, m);
}
HD double to_f(const Num& x, uint32_t& err) {          // float(x)
  if (!x.isint) return x.f;
  bool ovf = false;
  const double v = round_mag(x.m.w, false, 0, ovf);
  if (ovf && !err) err = E_OVERFLOW;      // int too large to convert to float
  return x.neg ? -v : v;
}
HD bool is_zero(const Num& x) { return x.isint ? mag_zero(x.m) : x.f == 0.0; }
HD bool truth(const Num& x) { return x.isint ? !mag_zero(x.m) : x.f != 0.0; }
HD Num from_bool(bool b) { return from_int(false, mag_small(b ? 1u : 0u)); }
HD Num neg(const Num& x) {
  if (!x.isint) return from_f(-x.f);
  return from_int(!x.neg, x.m);
}
HD Num int_add(bool an, const Mag& a, bool bn, const Mag& b, uint32_t& err) {
  if (an == bn) {
    bool ovf = false;
    const Mag s = mag_add(a, b, ovf);
    if (ovf && !err) err = E_RANGE;
    return from_int(an, s);
  }
  const int c = mag_cmp(a, b);
  if (c == 0) return from_int(false, mag_small(0));
  return c > 0 ? from_int(an, mag_sub(a, b)) : from_int(bn, mag_sub(b, a));
}
HD Num add(const Num& a, const Num& b, uint32_t& err) {
  if (a.isint && b.isint) return int_add(a.neg, a.m, b.neg, b.m, err);
  const double x = to_f(a, err), y = to_f(b, err);
  return from_f(x + y);
}
HD Num sub(const Num& a, const Num& b, uint32_t& err) {
  if (a.isint && b.isint) return int_add(a.neg, a.m, !b.neg, b.m, err);
  const double x = to_f(a, err), y = to_f(b, err);
  return from_f(x - y);
}
HD Num mul(const Num& a, const Num& b, uint32_t& err) {
  if (a.isint && b.isint) {
    bool ovf = false;
    const Mag p = mag_mul(a.m, b.m, ovf);
    if (ovf && !err) err = E_RANGE;
    return from_int(a.neg != b.neg, p);
  }
  const double x = to_f(a, err), y = to_f(b, err);
  return from_f(x * y);
}
// int / int, b != 0 (CPython long_true_divide: the exact ratio rounded once;
// OverflowError past the float range)
HD Num int_truediv(const Num& a, const Num& b, uint32_t& err) {
  const bool sgn = a.neg != b.neg;
  // a << s and b << (56 - s): up to 2 kLimbs + 2 limbs
  constexpr int W = 2 * kLimbs + 2;
  uint64_t n[W], d[W];
  for (int i = 0; i < W; ++i) {
    n[i] = i < kLimbs ? a.m.w[i] : 0;
    d[i] = i < kLimbs ? b.m.w[i] : 0;
  }
  const int na = bitlen(n), nb = bitlen(d);
  double q;
  bool ovf = false;
  if (na == 0) {
    q = 0.0;
  } else if (na <= 53 && nb <= 53) {      // CPython's fast path: one rounding
    q = (double)n[0] / (double)d[0];
  } else {
    // Q = floor(a * 2^s / b) has 55 or 56 bits; the remainder is the sticky
    const int s = 55 - (na - nb);
    auto shl = [](uint64_t (&v)[W], int k) {
      if (k <= 0) return;
      const int limbs = k >> 6, sh = k & 63;
      for (int i = W - 1; i >= 0; --i) {
        uint64_t x = i - limbs >= 0 ? v[i - limbs] << sh : 0;
        if (sh && i - limbs - 1 >= 0) x |= v[i - limbs - 1] >> (64 - sh);
        v[i] = x;
      }
    };
    shl(n, s > 0 ? s : 0);
    shl(d, s < 0 ? -s : 0);
    uint64_t Q[1] = {0};
    uint64_t t[W];
    for (int bit = 56; bit >= 0; --bit) {
      for (int i = 0; i < W; ++i) t[i] = d[i];
      shl(t, bit);
      int c = 0;                          // compare n with t
      for (int i = W - 1; i >= 0 && !c; --i)
        if (n[i] != t[i]) c = n[i] < t[i] ? -1 : 1;
      if (c >= 0) {
        uint64_t br = 0;
        for (int i = 0; i < W; ++i) {
          const uint64_t dd = n[i] - t[i];
          const uint64_t b1 = n[i] < t[i];
          n[i] = dd - br;
          br = b1 | (dd < br);
        }
        Q[0] |= 1ull << bit;
      }
    }
    bool sticky = false;
    for (int i = 0; i < W; ++i) sticky |= n[i] != 0;
    q = round_mag(Q, sticky, -s, ovf);
  }
  if (ovf && !err) err = E_OVERFLOW;      // integer division result too large
  return from_f(sgn ? -q : q);
}
// protectedDiv(a, b) = a / b, 1 on ZeroDivisionError: int / int checks b
// first; a float division converts both operands (either may overflow) and
// then checks b == 0 (CPython float_div)
HD Num pdiv(const Num& a, const Num& b, uint32_t& err) {
  if (a.isint && b.isint) return is_zero(b) ? from_bool(true) : int_truediv(a, b, err);
  const double x = to_f(a, err), y = to_f(b, err);
  return y == 0.0 ? from_bool(true) : from_f(x / y);
}
// Python's comparison of two numbers: -1, 0, 1, or 2 (unordered: a nan)
HD int cmp(const Num& a, const Num& b) {
  if (!a.isint && !b.isint) {
    if (a.f < b.f) return -1;
    if (a.f > b.f) return 1;
    return a.f == b.f ? 0 : 2;
  }
  if (a.isint && b.isint) {
    if (a.neg != b.neg) return a.neg ? -1 : 1;
    const int c = mag_cmp(a.m, b.m);
    return a.neg ? -c : c;
  }
  // int vs float, exactly (CPython float_richcompare)
  const bool swap = !a.isint;
  const Num& i = swap ? b : a;
  const double f = swap ? a.f : b.f;
  int r;
  if (f != f) return 2;
  if (__builtin_isinf(f)) {
    r = f > 0 ? -1 : 1;
  } else {
    const int isg = mag_zero(i.m) ? 0 : (i.neg ? -1 : 1);
    const int fsg = f > 0 ? 1 : f < 0 ? -1 : 0;
    if (isg != fsg) {
      r = isg < fsg ? -1 : 1;
    } else if (isg == 0) {
      r = 0;
    } else {
      // |f|'s integer part exactly (|f| < 2^1024 fits the magnitude)
      const double af = __builtin_fabs(f);
      int e;
      const double fr = frexp(af, &e);              // af = fr * 2^e
      const uint64_t mant = (uint64_t)ldexp(fr, 53);
      Mag ip = mag_small(0);
      bool frac = false;
      const int sh = e - 53;
      if (sh >= 0) {
        ip.w[sh >> 6] = mant << (sh & 63);
        if ((sh & 63) && (sh >> 6) + 1 < kLimbs) ip.w[(sh >> 6) + 1] = mant >> (64 - (sh & 63));
      } else if (-sh < 64) {
        ip.w[0] = mant >> -sh;
        frac = (mant & ((1ull << -sh) - 1)) != 0;
      } else {
        frac = mant != 0;
      }
      int c = mag_cmp(i.m, ip);
      if (c == 0 && frac) c = -1;                   // |i| = floor(|f|) < |f|
      r = isg > 0 ? c : -c;
    }
  }
  return swap ? -r : r;
}

// One F program on one case with Python-number semantics (f_run's opcode
// set minus numpy's).  xv(v): the case's variable v.  err: the first error
// (E_*); evaluation stops there, as the reference's exception ends the case.
// Returns false on an opcode outside that set (gpe_load_exact rejects such
// programs first).
template <int D, class XV>
HD bool run(const uint32_t* W, const uint32_t* ints, XV xv, Num& T, uint32_t& err) {
  Num stk[D];
  T = from_f(0.0);
  err = E_NONE;
  // an int constant (index field 1): its row of the int table in the two
  // data words; otherwise the double's bits
  auto konst = [&](uint32_t w, const uint32_t* p) -> Num {
    if (w >> 16) return from_words(ints + kWords * ((size_t)p[0] | ((size_t)p[1] << 32)));
    return from_f(dbits(p[0], p[1]));
  };
  uint32_t i = 0;
  for (;;) {
    if (err) return true;
    const uint32_t w = W[i++];
    const uint32_t op = w & 0xffu, d = (w >> 8) & 0xffu, x = w >> 16;
    if (op == OP_END) return true;
    if (op == OP_LDV) { T = from_f(xv(x)); continue; }
    if (op == OP_LDC) { T = konst(w, W + i); i += 2; continue; }
    if (op == OP_PUSH) { stk[d] = T; continue; }
    if (op == OP_PUSHV) { stk[d] = T; T = from_f(xv(x)); continue; }
    if (op == OP_PUSHC) { stk[d] = T; T = konst(w, W + i); i += 2; continue; }
    if (op == OP_NEG) { T = neg(T); continue; }
    if (op == OP_SIN || op == OP_COS) {
      const double v = to_f(T, err);     // math.sin(int): float(int) first
      if (err) return true;
      if (__builtin_isinf(v)) err = E_VALUE;
      T = from_f(glibc_trig(v, op == OP_COS));
      continue;
    }
    if (op == OP_NOT) { T = from_bool(!truth(T)); continue; }
    if (op == OP_ITE) { T = truth(stk[d]) ? stk[d + 1] : T; continue; }
    if (op < OP_ADD || op >= OP_XOR) return false;
    const uint32_t fam = (op - OP_ADD) / 3, form = (op - OP_ADD) % 3;
    Num a;
    if (form == 0) a = stk[d];
    else if (form == 1) a = from_f(xv(x));
    else { a = konst(w, W + i); i += 2; }
    const Num& b = T;
    switch (fam) {
      case 0: T = add(a, b, err); break;
      case 1: T = sub(a, b, err); break;                  // a - T
      case 2: T = sub(b, a, err); break;                  // T - a
      case 3: T = mul(a, b, err); break;
      case 4: T = pdiv(a, b, err); break;                 // pdiv(a, T)
      case 5: T = pdiv(b, a, err); break;                 // pdiv(T, a)
      case 6: T = from_bool(cmp(a, b) == -1); break;      // a < T
      case 7: T = from_bool(cmp(b, a) == -1); break;      // T < a
      case 8: T = from_bool(cmp(a, b) == 0); break;
      case 9: T = from_bool(truth(a) && truth(b)); break;
      default: T = from_bool(truth(a) || truth(b)); break;
    }
  }
}
}  // namespace xint
static_assert(xint::kWords == GPE_XINT_WORDS && xint::E_RANGE == GPE_ERR_XINT_RANGE &&
                  xint::E_VALUE == GPE_ERR_VALUE && xint::E_OVERFLOW == GPE_ERR_OVERFLOW,
              "include/gpeval.h and the exact pass agree");

// ------------------------------------------------------- host big ints --
// The exact pass's programs past the device's 1088 bits (bigint_host.h: an
// int constant at or past 2^1087, or a case the device ended with E_RANGE):
// the host evaluates them with xint::run's semantics and no size limit.  The
// int table as the host keeps it: variable-length rows of two's complement
// words (row r = words[off[r] .. off[r + 1])).
#include "bigint_host.h"
namespace hbig {
static_assert(E_VALUE == xint::E_VALUE && E_OVERFLOW == xint::E_OVERFLOW, "one error code set");
struct Rows {
  const uint32_t* words;
  const int64_t* off;
  int64_t n;
};
// One F program on one case (xint::run with unbounded ints).  Returns false
// on an opcode outside the exact pass's set or an int row out of range.
template <class XV>
bool run(const uint32_t* W, const Rows& ints, XV xv, Num& T, uint32_t& err) {
  Num stk[32];
  T = from_f(0.0);
  err = E_NONE;
  bool ok = true;
  auto konst = [&](uint32_t w, const uint32_t* p) -> Num {
    if (w >> 16) {
      const uint64_t r = (uint64_t)p[0] | ((uint64_t)p[1] << 32);
      if (r >= (uint64_t)ints.n) {
        ok = false;
        return from_f(0.0);
      }
      return from_words(ints.words + ints.off[r], ints.off[r + 1] - ints.off[r]);
    }
    return from_f(dbits(p[0], p[1]));
  };
  uint32_t i = 0;
  for (;;) {
    if (err || !ok) return ok;
    const uint32_t w = W[i++];
    const uint32_t op = w & 0xffu, d = (w >> 8) & 0xffu, x = w >> 16;
    if (d >= 32 || (op == OP_ITE && d >= 31)) return false;
    if (op == OP_END) return true;
    if (op == OP_LDV) { T = from_f(xv(x)); continue; }
    if (op == OP_LDC) { T = konst(w, W + i); i += 2; continue; }
    if (op == OP_PUSH) { stk[d] = T; continue; }
    if (op == OP_PUSHV) { stk[d] = std::move(T); T = from_f(xv(x)); continue; }
    if (op == OP_PUSHC) { stk[d] = std::move(T); T = konst(w, W + i); i += 2; continue; }
    if (op == OP_NEG) { T = neg(T); continue; }
    if (op == OP_SIN || op == OP_COS) {
      const double v = to_f(T, err);     // math.sin(int): float(int) first
      if (err) return true;
      if (__builtin_isinf(v)) err = E_VALUE;
      T = from_f(glibc_trig(v, op == OP_COS));
      continue;
    }
    if (op == OP_NOT) { T = from_bool(!truth(T)); continue; }
    if (op == OP_ITE) { T = truth(stk[d]) ? stk[d + 1] : T; continue; }
    if (op < OP_ADD || op >= OP_XOR) return false;
    const uint32_t fam = (op - OP_ADD) / 3, form = (op - OP_ADD) % 3;
    Num a;
    if (form == 0) a = stk[d];
    else if (form == 1) a = from_f(xv(x));
    else { a = konst(w, W + i); i += 2; }
    const Num& b = T;
    Num r;
    switch (fam) {
      case 0: r = add(a, b, err); break;
      case 1: r = sub(a, b, err); break;                  // a - T
      case 2: r = sub(b, a, err); break;                  // T - a
      case 3: r = mul(a, b, err); break;
      case 4: r = pdiv(a, b, err); break;                 // pdiv(a, T)
      case 5: r = pdiv(b, a, err); break;                 // pdiv(T, a)
      case 6: r = from_bool(cmp(a, b) == -1); break;      // a < T
      case 7: r = from_bool(cmp(b, a) == -1); break;      // T < a
      case 8: r = from_bool(cmp(a, b) == 0); break;
      case 9: r = from_bool(truth(a) && truth(b)); break;
      default: r = from_bool(truth(a) || truth(b)); break;
    }
    T = std::move(r);
  }
}
}  // namespace hbig

}  // namespace
