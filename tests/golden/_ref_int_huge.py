#!/usr/bin/env python3
"""Ints past the device's 1088 bits, pinned: trees whose Python ints (exact,
unbounded: ``gp.compile``'s ``eval``, deap/gp.py:462-487; protectedDiv's int
1 per case, examples/gp/symbreg.py:29-33) grow past 2**1088 and then cancel,
divide exactly, compare, or overflow only where the error formula
(``symbreg.py:60-61``) converts them to float — evaluated by the REFERENCE
on the C1 points.  The exact-integer pass evaluates such programs on the
host with unbounded ints (csrc/bigint_host.h); tests/test_gpu.py checks its
fitness and exception types against these.

    h = (2**400 + 1)**3            per case: add(2**400, protectedDiv(x, sub(x, x)))
    sub(h, h)                      0: the fitness of the zero function
    protectedDiv(h, h)             1.0: int / int, the exact ratio rounded once
    protectedDiv(h, add(h, 1))     1.0 (rounded from 1 - 2**-1200)
    sub(h, 1)                      OverflowError: float(h) in the formula
    sub(add(C, one), C)            1 with C = 2**1200 folded to one constant

Build container only: ``python3 tests/golden/_ref_int_huge.py`` (needs the
2to3 copy from ``make_oracle_copy.sh``; writes ``c1_int_huge.json.gz``).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (imports the reference copy)
from make_golden import datasets, gp  # noqa: E402
from _ref_int_residual import power_of_two  # noqa: E402


def main():
    pset1 = mg.arith_pset(1, True)
    X1, T1 = datasets.symbreg_points()
    one = "protectedDiv(x, sub(x, x))"                      # int 1 per case
    b400 = "add(%s, %s)" % (power_of_two(400), one)         # 2**400 + 1
    h = "mul(mul(%s, %s), %s)" % (b400, b400, b400)         # ~2**1200
    c1200 = power_of_two(1200)                              # folds to one int
    trees = [
        "sub(%s, %s)" % (h, h),                             # cancel: 0
        "add(sub(%s, %s), x)" % (h, h),                     # x
        "protectedDiv(%s, %s)" % (h, h),                    # exactly 1.0
        "protectedDiv(%s, add(%s, 1))" % (h, h),            # 1.0, rounded
        "protectedDiv(add(%s, %s), %s)" % (h, one, h),      # 1.0, rounded
        "mul(x, protectedDiv(%s, mul(%s, add(1, 1))))" % (h, h),   # x / 2
        "sub(mul(mul(%s, %s), %s), 1)" % (b400, b400, b400),   # OverflowError
        "protectedDiv(x, %s)" % h,                          # OverflowError
        "sub(add(%s, %s), %s)" % (c1200, one, c1200),       # 1: a wide constant
        "mul(sub(add(%s, %s), %s), x)" % (c1200, one, c1200),      # x
        "protectedDiv(%s, %s)" % (h, power_of_two(1100)),   # ~2**100
    ]
    mg.symreg_fixture("c1_int_huge", pset1, trees, X1, T1,
                      {"pset": "symbreg", "data": {"kind": "symbreg_points"}})
    for s in trees:
        f = gp.compile(s, pset1)
        try:
            print(len(s), f(0.5))
        except OverflowError as exc:
            print(len(s), "OverflowError", exc)


if __name__ == "__main__":
    main()
