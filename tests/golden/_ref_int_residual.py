#!/usr/bin/env python3
"""The integer residual, pinned: trees where Python's exact integers beyond
2**53 meet a per-case integer (``protectedDiv``'s zero branch returns int 1,
examples/gp/symbreg.py:29-33), evaluated by the REFERENCE (``gp.compile`` +
the ``symbreg.py:60-61`` loop) on the C1 points.  Round 3 adds ints up to
2**200, a product of two per-case ints, int / int ratios, a per-case value
that is an int at one point (x = 0) and a float elsewhere, and sin/cos/neg
of exact ints.

    sub(add(BIG, protectedDiv(x, sub(x, x))), BIG)

is 1 for every case in Python (``BIG + 1 - BIG`` in exact integers); a device
that folds BIG to float64 computes ``(fl(BIG) + 1.0) - fl(BIG)``, 0 for BIG =
2**54 + 2.  The evaluator re-evaluates such individuals in the device's
exact-integer pass (``gpe_load_exact``); tests/test_gpu.py checks it
against these values.

Build container only: ``python3 tests/golden/_ref_int_residual.py`` (needs
the 2to3 copy from ``make_oracle_copy.sh``; writes ``c1_int_residual.json.gz``).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (imports the reference copy)
from make_golden import datasets, gp  # noqa: E402


def power_of_two(k):
    """An int-only subtree worth 2**k (k >= 1) over add/mul of the literal 1."""
    parts, bit, sq = [], 0, "add(1, 1)"
    while k:
        if k & 1:
            parts.append(sq)
        k >>= 1
        bit += 1
        sq = "mul(%s, %s)" % (sq, sq)
    out = parts[0]
    for p in parts[1:]:
        out = "mul(%s, %s)" % (out, p)
    return out


def main():
    pset1 = mg.arith_pset(1, True)
    X1, T1 = datasets.symbreg_points()
    big = "add(%s, add(1, 1))" % power_of_two(54)           # 2**54 + 2
    big2 = "add(%s, 1)" % power_of_two(60)                  # 2**60 + 1
    per_case_one = "protectedDiv(x, sub(x, x))"             # int 1 per case
    p30, p60 = power_of_two(30), power_of_two(60)
    b80 = "add(%s, add(1, add(1, 1)))" % power_of_two(80)   # 2**80 + 3
    b120 = "add(%s, 1)" % power_of_two(120)                 # 2**120 + 1
    b200 = "add(%s, 1)" % power_of_two(200)                 # 2**200 + 1
    one_at_0 = "protectedDiv(1, x)"     # int 1 at x = 0.0, a float elsewhere
    trees = [
        "sub(add(%s, %s), %s)" % (big, per_case_one, big),
        "sub(add(%s, %s), %s)" % (big2, per_case_one, big2),
        "mul(x, sub(add(%s, %s), %s))" % (big, per_case_one, big),
        # round 3: 2**80 .. 2**200, two per-case ints multiplied, int / int
        # rounded once, a per-case int that is an int at one point only,
        # sin/cos and neg of exact ints
        "sub(add(%s, %s), %s)" % (b80, per_case_one, b80),
        "sub(add(%s, %s), %s)" % (b120, per_case_one, b120),
        "sub(add(%s, %s), %s)" % (b200, per_case_one, b200),
        "sub(mul(add(%s, %s), add(%s, %s)), %s)" % (p30, per_case_one, p30,
                                                    per_case_one, p60),
        "protectedDiv(add(%s, %s), add(add(1, 1), %s))" % (big, per_case_one,
                                                          per_case_one),
        "protectedDiv(sub(%s, %s), add(%s, %s))" % (b80, per_case_one, b120,
                                                    per_case_one),
        "sub(add(%s, %s), %s)" % (big, one_at_0, big),
        "add(mul(x, sub(add(%s, %s), %s)), cos(sub(add(%s, %s), %s)))"
        % (b120, per_case_one, b120, big, per_case_one, big),
        "neg(sin(sub(mul(add(%s, %s), %s), %s)))" % (p30, per_case_one, p30,
                                                     p60),
        "mul(sub(add(%s, %s), %s), x)" % (b80, one_at_0, b80),
        # control: the same shape below 2**53 is exact on the device too
        "sub(add(%s, %s), %s)" % (power_of_two(40), per_case_one,
                                   power_of_two(40)),
    ]
    mg.symreg_fixture("c1_int_residual", pset1, trees, X1, T1,
                      {"pset": "symbreg", "data": {"kind": "symbreg_points"}})
    for s in trees:
        f = gp.compile(s, pset1)
        print(len(s), f(0.5))


if __name__ == "__main__":
    main()
