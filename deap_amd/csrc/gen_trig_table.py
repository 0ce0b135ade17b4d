#!/usr/bin/env python3
"""Regenerate trig_table.json (needs mpmath; the build only reads the JSON).

sin/cos of j*pi/32 (j = 0..63) as double-doubles, pi/32 in three parts for the
Cody-Waite reduction, and the Taylor coefficients of the short polynomials
used on |r| <= pi/64 (see gp_trig in gpeval.hip)."""
import json
import os

import mpmath

mpmath.mp.prec = 300


def dd(v):
    h = float(v)
    return h, float(v - mpmath.mpf(h))


def main():
    c = mpmath.pi / 32
    c1 = float(c)
    c2 = float(c - c1)
    c3 = float(c - c1 - c2)
    rows = []
    for j in range(64):
        sh, sl = dd(mpmath.sin(j * c))
        ch, cl = dd(mpmath.cos(j * c))
        rows.append([sh, sl, ch, cl])
    for j in (0, 32):
        rows[j][0] = rows[j][1] = 0.0
    for j in (16, 48):
        rows[j][2] = rows[j][3] = 0.0
    f = mpmath.factorial
    out = {"C": [c1.hex(), c2.hex(), c3.hex()],
           "INV": float(32 / mpmath.pi).hex(),
           "Ps": [float((-1) ** (k + 1) / f(2 * k + 3)).hex() for k in range(4)],
           "Pc": [float((-1) ** k / f(2 * k + 4)).hex() for k in range(4)],
           "table": [[v.hex() for v in r] for r in rows]}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "trig_table.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0)


if __name__ == "__main__":
    main()
