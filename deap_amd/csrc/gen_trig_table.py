#!/usr/bin/env python3
"""Regenerate trig_table.json (needs mpmath; the build only reads the JSON).

The table-driven fp64 sin/cos of the interpreters (``gp_trig`` in gpeval.hip,
``Gen.trig_ops`` in gen_asm.py) works on a grid of step c = pi/256:

* ``table``: sin(j*c) as a double-double (hi, lo) for j = 0 .. 767, so that
  sin(x) reads entries j and j + 128 (= cos(j*c)) and cos(x) = sin(x + pi/2)
  reads j + 128 and j + 256, for j = k mod 512, without wrapping.  Exact
  zeros (j = 0, 256, 512) are stored as (0, 0).
* ``S1`` = c rounded to double, ``S2`` = c - S1 rounded: the fast reduction
  (|x| < 2^14, |k| < 2^21) is t = fma(-k, S1, x), exact — x - k*S1 is a
  multiple of 2^-60 (x >= c/2 has ulp >= 2^-60, k*S1 is a multiple of
  2^-59) below 2^-7 in magnitude, so it fits 53 bits — and rl = k*(-S2)
  (|rl| < 2^-40, error < 2^-92).
* ``C``: c as three doubles C1 + C2 + C3 (the long reduction, |x| >= 2^14).
* ``INV`` = 256/pi; ``Ps``/``Pc``: Taylor coefficients of
  (sin r - r)/r^3 and (cos r - 1)/r^2 in z = r^2 (three each; the first Pc
  coefficient is -1/2 exactly), enough for |r| <= pi/512.

Tables of ``glibc_sin``/``glibc_cos`` (gpeval.hip: the reference's own libm,
glibc 2.35 ``sysdeps/ieee754/dbl-64/s_sin.c`` + ``branred.c``, restated):

* ``glibc_sincostab``: sin and cos of i/128, i < 110, each as a
  double-double (sn, ssn, cs, ccs) — glibc's ``__sincostab``;
* ``glibc_toverp``: 2/pi in 75 base-2^24 digits — ``branred.h``'s
  ``toverp``.
Both are generated here from their definitions; ``tests/test_lib.py`` pins
the restatement to the host's libm bit for bit.
"""
import json
import os
from fractions import Fraction

import mpmath

mpmath.mp.prec = 400
N = 256                                  # grid steps per pi
ENTRIES = 3 * N                          # j + 256 < 768 for j < 512


def dd(v):
    h = float(v)
    return h, float(v - mpmath.mpf(h))


def round_bits(v, bits):
    """Fraction v rounded to ``bits`` significant bits (nearest)."""
    e = v.numerator.bit_length() - v.denominator.bit_length()
    if Fraction(2) ** e > abs(v):
        e -= 1
    scale = Fraction(2) ** (bits - 1 - e)
    r = Fraction(round(v * scale)) / scale
    assert (r * scale).denominator == 1
    return r


def main():
    c = mpmath.pi / N
    cf = Fraction(int(mpmath.floor(c * mpmath.mpf(2) ** 420)), 2 ** 420)
    s1 = round_bits(cf, 53)
    s2 = float(cf - s1)
    c1 = float(cf)
    c2 = float(cf - Fraction(c1))
    c3 = float(cf - Fraction(c1) - Fraction(c2))
    rows = []
    for j in range(ENTRIES):
        if j % N == 0:
            rows.append((0.0, 0.0))
        else:
            rows.append(dd(mpmath.sin(j * c)))
    gtab = []
    for i in range(110):
        x = mpmath.mpf(i) / 128
        gtab += list(dd(mpmath.sin(x))) + list(dd(mpmath.cos(x)))
    with mpmath.workprec(2400):                 # 75 x 24 bits of 2/pi
        v = 2 / mpmath.pi
        toverp = []
        for _ in range(75):
            v *= 2 ** 24
            d = int(mpmath.floor(v))
            toverp.append(d)
            v -= d
    f = mpmath.factorial
    out = {"N": N,
           "glibc_sincostab": [v.hex() for v in gtab],
           "glibc_toverp": toverp,
           "INV": float(N / mpmath.pi).hex(),
           "S1": float(s1).hex(), "S2": s2.hex(),
           "C": [c1.hex(), c2.hex(), c3.hex()],
           "Ps": [float(-1 / f(3)).hex(), float(1 / f(5)).hex(),
                  float(-1 / f(7)).hex()],
           "Pc": [float(-1 / f(2)).hex(), float(1 / f(4)).hex(),
                  float(-1 / f(6)).hex()],
           "table": [[a.hex(), b.hex()] for a, b in rows]}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "trig_table.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0)


if __name__ == "__main__":
    main()
