// bigint_host.h — Python ints without a size limit, for the exact-integer
// pass's programs that the device's 1088-bit magnitudes (gpeval.hip namespace
// xint) cannot hold: an int constant at or past 2^1087, or an int that the
// evaluation grows past 2^1088 (the device ends such a case with E_RANGE).
// The reference keeps going with unbounded ints (deap/gp.py:462-487 `eval`
// of the compiled tree; examples/gp/symbreg.py:29-33 protectedDiv's int 1):
// those cancel (sub(h, h)), divide exactly (int / int rounds the exact ratio
// once, CPython long_true_divide) or overflow only where they convert to
// float.  This is the host evaluator of those programs, operation for
// operation xint's semantics with a limb vector instead of 17 fixed limbs.
//
// Included by gpeval.hip after namespace xint (it uses the opcodes, dbits and
// glibc_trig defined there).  Magnitudes are little-endian 64-bit limbs
// without a high zero limb (0 is the empty vector); bit counts are int64.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace hbig {

using Mag = std::vector<uint64_t>;

inline void trim(Mag& a) {
  while (!a.empty() && !a.back()) a.pop_back();
}
inline int mag_cmp(const Mag& a, const Mag& b) {
  if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
  for (size_t i = a.size(); i-- > 0;)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}
inline Mag mag_add(const Mag& a, const Mag& b) {
  const Mag& x = a.size() >= b.size() ? a : b;
  const Mag& y = a.size() >= b.size() ? b : a;
  Mag r(x.size() + 1);
  uint64_t c = 0;
  for (size_t i = 0; i < x.size(); ++i) {
    const uint64_t yi = i < y.size() ? y[i] : 0;
    const uint64_t s = x[i] + c;
    const uint64_t c1 = s < c;
    r[i] = s + yi;
    c = c1 | (r[i] < s);
  }
  r[x.size()] = c;
  trim(r);
  return r;
}
inline Mag mag_sub(const Mag& a, const Mag& b) {       // a >= b
  Mag r(a.size());
  uint64_t br = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    const uint64_t bi = i < b.size() ? b[i] : 0;
    const uint64_t d = a[i] - bi;
    const uint64_t b1 = a[i] < bi;
    r[i] = d - br;
    br = b1 | (d < br);
  }
  trim(r);
  return r;
}
inline Mag mag_mul(const Mag& a, const Mag& b) {
  if (a.empty() || b.empty()) return Mag();
  Mag p(a.size() + b.size(), 0);
  for (size_t i = 0; i < a.size(); ++i) {
    uint64_t carry = 0;
    for (size_t j = 0; j < b.size(); ++j) {
      const unsigned __int128 t = (unsigned __int128)a[i] * b[j] + p[i + j] + carry;
      p[i + j] = (uint64_t)t;
      carry = (uint64_t)(t >> 64);
    }
    p[i + b.size()] = carry;
  }
  trim(p);
  return p;
}
inline Mag mag_shl(const Mag& a, int64_t k) {           // a * 2^k, k >= 0
  if (a.empty() || k <= 0) return a;
  const int64_t limbs = k >> 6;
  const int sh = (int)(k & 63);
  Mag r((size_t)limbs + a.size() + 1, 0);
  for (size_t i = 0; i < a.size(); ++i) {
    r[(size_t)limbs + i] |= a[i] << sh;
    if (sh) r[(size_t)limbs + i + 1] |= a[i] >> (64 - sh);
  }
  trim(r);
  return r;
}
inline int64_t bitlen(const Mag& a) {
  return a.empty() ? 0 : 64 * (int64_t)(a.size() - 1) + (64 - __builtin_clzll(a.back()));
}
inline int bit_at(const Mag& a, int64_t b) {
  if (b < 0 || b >= 64 * (int64_t)a.size()) return 0;
  return (int)((a[(size_t)(b >> 6)] >> (b & 63)) & 1u);
}
inline bool any_below(const Mag& a, int64_t b) {        // a bit < b set
  for (size_t i = 0; i < a.size() && 64 * (int64_t)i < b; ++i) {
    const int64_t k = b - 64 * (int64_t)i;
    const uint64_t mask = k >= 64 ? ~0ull : ((1ull << k) - 1);
    if (a[i] & mask) return true;
  }
  return false;
}
inline uint64_t bits_from(const Mag& a, int64_t b) {    // 64 bits from bit b
  const size_t i = (size_t)(b >> 6);
  const int sh = (int)(b & 63);
  uint64_t lo = i < a.size() ? a[i] >> sh : 0;
  if (sh && i + 1 < a.size()) lo |= a[i + 1] << (64 - sh);
  return lo;
}
// round-to-nearest-even of (a + sticky * tiny) * 2^e2 to a double, as
// CPython's float(int) and int / int round (xint::round_mag)
inline double round_mag(const Mag& w, bool sticky, int64_t e2, bool& ovf) {
  const int64_t nb = bitlen(w);
  if (nb == 0) return 0.0;
  const int64_t p = nb - 1 + e2;
  if (p >= 1024) {
    ovf = true;
    return __builtin_inf();
  }
  const int64_t keep = p >= -1022 ? 53 : p + 1075;
  const int64_t sh = nb - keep;
  if (sh <= 0) return ldexp((double)w[0], (int)e2);     // nb <= 53: exact
  uint64_t mant = keep > 0 ? bits_from(w, sh) & ((1ull << keep) - 1) : 0;
  const int rb = bit_at(w, sh - 1);
  const bool rest = sticky || any_below(w, sh - 1);
  if (rb && (rest || (mant & 1u))) ++mant;
  const double v = ldexp((double)mant, (int)(sh + e2));
  ovf |= __builtin_isinf(v);
  return v;
}

struct Num {
  bool isint = false;
  bool neg = false;            // ints: sign (never set on 0)
  double f = 0.0;
  Mag m;
};
inline Num from_f(double f) {
  Num r;
  r.f = f;
  return r;
}
inline Num from_int(bool neg, Mag m) {
  Num r;
  r.isint = true;
  r.neg = neg && !m.empty();
  r.m = std::move(m);
  return r;
}
inline Num from_bool(bool b) { return from_int(false, b ? Mag{1} : Mag()); }
// n little-endian 32-bit words, two's complement (the exact table's rows)
inline Num from_words(const uint32_t* w, int64_t n) {
  Mag m((size_t)((n + 1) / 2), 0);
  for (int64_t i = 0; i < n; ++i) m[(size_t)(i / 2)] |= (uint64_t)w[i] << (32 * (i & 1));
  const bool neg = n > 0 && (w[n - 1] >> 31) != 0;
  if (neg) {
    if (n & 1) m.back() |= 0xffffffff00000000ull;      // sign-extend the odd word
    uint64_t c = 1;
    for (auto& x : m) {
      x = ~x + c;
      c = c && x == 0;
    }
  }
  trim(m);
  return from_int(neg, std::move(m));
}
enum : uint32_t { E_NONE = 0, E_VALUE = 1, E_OVERFLOW = 2 };
inline double to_f(const Num& x, uint32_t& err) {      // float(x)
  if (!x.isint) return x.f;
  bool ovf = false;
  const double v = round_mag(x.m, false, 0, ovf);
  if (ovf && !err) err = E_OVERFLOW;
  return x.neg ? -v : v;
}
inline bool truth(const Num& x) { return x.isint ? !x.m.empty() : x.f != 0.0; }
inline Num neg(const Num& x) { return x.isint ? from_int(!x.neg, x.m) : from_f(-x.f); }
inline Num int_add(bool an, const Mag& a, bool bn, const Mag& b) {
  if (an == bn) return from_int(an, mag_add(a, b));
  const int c = mag_cmp(a, b);
  if (c == 0) return from_int(false, Mag());
  return c > 0 ? from_int(an, mag_sub(a, b)) : from_int(bn, mag_sub(b, a));
}
inline Num add(const Num& a, const Num& b, uint32_t& err) {
  if (a.isint && b.isint) return int_add(a.neg, a.m, b.neg, b.m);
  const double x = to_f(a, err), y = to_f(b, err);
  return from_f(x + y);
}
inline Num sub(const Num& a, const Num& b, uint32_t& err) {
  if (a.isint && b.isint) return int_add(a.neg, a.m, !b.neg, b.m);
  const double x = to_f(a, err), y = to_f(b, err);
  return from_f(x - y);
}
inline Num mul(const Num& a, const Num& b, uint32_t& err) {
  if (a.isint && b.isint) return from_int(a.neg != b.neg, mag_mul(a.m, b.m));
  const double x = to_f(a, err), y = to_f(b, err);
  return from_f(x * y);
}
// int / int, b != 0: the exact ratio rounded once (CPython long_true_divide)
inline Num int_truediv(const Num& a, const Num& b, uint32_t& err) {
  const bool sgn = a.neg != b.neg;
  const int64_t na = bitlen(a.m), nb = bitlen(b.m);
  double q;
  bool ovf = false;
  if (na == 0) {
    q = 0.0;
  } else if (na <= 53 && nb <= 53) {       // CPython's fast path: one rounding
    q = (double)a.m[0] / (double)b.m[0];
  } else {
    // Q = floor(a * 2^s / b) has 55 or 56 bits; the remainder is the sticky
    const int64_t s = 55 - (na - nb);
    Mag n = mag_shl(a.m, s > 0 ? s : 0);
    const Mag d = mag_shl(b.m, s < 0 ? -s : 0);
    uint64_t Q = 0;
    for (int bit = 56; bit >= 0; --bit) {
      const Mag t = mag_shl(d, bit);
      if (mag_cmp(n, t) >= 0) {
        n = mag_sub(n, t);
        Q |= 1ull << bit;
      }
    }
    q = round_mag(Mag{Q}, !n.empty(), -s, ovf);
  }
  if (ovf && !err) err = E_OVERFLOW;
  return from_f(sgn ? -q : q);
}
// protectedDiv(a, b): a / b, 1 on ZeroDivisionError (xint::pdiv)
inline Num pdiv(const Num& a, const Num& b, uint32_t& err) {
  if (a.isint && b.isint) return b.m.empty() ? from_bool(true) : int_truediv(a, b, err);
  const double x = to_f(a, err), y = to_f(b, err);
  return y == 0.0 ? from_bool(true) : from_f(x / y);
}
// Python's comparison of two numbers: -1, 0, 1, or 2 (a nan)
inline int cmp(const Num& a, const Num& b) {
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
  const bool swap = !a.isint;              // int vs float, exactly
  const Num& i = swap ? b : a;
  const double f = swap ? a.f : b.f;
  int r;
  if (f != f) return 2;
  if (__builtin_isinf(f)) {
    r = f > 0 ? -1 : 1;
  } else {
    const int isg = i.m.empty() ? 0 : (i.neg ? -1 : 1);
    const int fsg = f > 0 ? 1 : f < 0 ? -1 : 0;
    if (isg != fsg) {
      r = isg < fsg ? -1 : 1;
    } else if (isg == 0) {
      r = 0;
    } else {
      int e;
      const double fr = frexp(__builtin_fabs(f), &e);  // |f| = fr 2^e
      const uint64_t mant = (uint64_t)ldexp(fr, 53);
      Mag ip;
      bool frac = false;
      const int sh = e - 53;
      if (sh >= 0) {
        ip = mag_shl(Mag{mant}, sh);
      } else if (-sh < 64) {
        ip = Mag{mant >> -sh};
        trim(ip);
        frac = (mant & ((1ull << -sh) - 1)) != 0;
      } else {
        frac = mant != 0;
      }
      int c = mag_cmp(i.m, ip);
      if (c == 0 && frac) c = -1;          // |i| = floor(|f|) < |f|
      r = isg > 0 ? c : -c;
    }
  }
  return swap ? -r : r;
}

}  // namespace hbig
