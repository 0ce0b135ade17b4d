#!/usr/bin/env python3
"""The integer residual, pinned: trees where Python's exact integers beyond
2**53 meet a per-case integer (``protectedDiv``'s zero branch returns int 1,
examples/gp/symbreg.py:29-33), evaluated by the REFERENCE (``gp.compile`` +
the ``symbreg.py:60-61`` loop) on the C1 points.

    sub(add(BIG, protectedDiv(x, sub(x, x))), BIG)

is 1 for every case in Python (``BIG + 1 - BIG`` in exact integers); a device
that folds BIG to float64 computes ``(fl(BIG) + 1.0) - fl(BIG)``, 0 for BIG =
2**54 + 2.  The evaluator warns for such individuals
(``evaluator.py: _warn_inexact``); tests/test_gpu.py records the divergence
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
    trees = [
        "sub(add(%s, %s), %s)" % (big, per_case_one, big),
        "sub(add(%s, %s), %s)" % (big2, per_case_one, big2),
        "mul(x, sub(add(%s, %s), %s))" % (big, per_case_one, big),
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
