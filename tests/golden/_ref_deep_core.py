#!/usr/bin/env python3
"""The deep asm core, pinned: C4-pset programs that need 6..12 operand-stack
slots (the deep core's range), with sin/cos, some of them
on the glibc redo path (a sin/cos argument at or past 2^40), evaluated by the
REFERENCE (``gp.compile`` and the ``examples/gp/symbreg.py:60-61`` loop
shape) at 4,096 C4 cases (target from ``benchmarks/gp.py:60-72``,
``unwrapped_ball``).

A tree needing s slots is a full binary tree of depth s over the C4
binary primitives (sin/cos/neg wrapped around some inner nodes) whose leaves
are height-1 trees over a variable from the reference's own ``gp.genFull``
under a fixed seed; the slot count (the flattener's Sethi-Ullman need) is
checked per tree, and a tree whose constant folds lower it is redrawn.  The redo-path
trees combine such a tree with ``sin(protectedDiv(protectedDiv(ARGa,
sub(ARGb, ARGc)), sub(ARGd, ARGe)))``: the nested ratios of near-equal cases
reach 2^40 at some of the 4,096 cases.

Build container only: ``python3 tests/golden/_ref_deep_core.py`` (needs the
2to3 copy from ``make_oracle_copy.sh``; writes ``c4_deep_core.json.gz``).
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (imports the reference copy)
from make_golden import datasets, gp  # noqa: E402

from deap_amd import configs  # noqa: E402
from deap_amd import gp as dgp  # noqa: E402
from deap_amd.flatten import Flattener  # noqa: E402

N_CASES, SEED = 4096, 77
# slots 6..12, most at 6..8 (a tree at s slots has >= 2^(s+1) leaves)
PLAN = [6] * 150 + [7] * 70 + [8] * 24 + [9] * 6 + [10] * 3 + [11] * 2 + [12]
N_REDO = 32


def skeleton(pset, rng, s):
    """A tree needing s + 1 stack slots: a full binary tree of depth s + 1
    over leaves that are primitives themselves (the Strahler number that
    forces s + 1 pushes), inner nodes from the C4 binary primitives,
    about a third of its inner nodes wrapped in sin/cos/neg, leaves drawn
    by the reference's own gp.genFull (height 1, over a variable)."""
    if s < 0:                             # a primitive over a variable
        while True:
            leaf = str(gp.PrimitiveTree(gp.genFull(pset, min_=1, max_=1)))
            if "ARG" in leaf:
                return leaf
    left, right = skeleton(pset, rng, s - 1), skeleton(pset, rng, s - 1)
    out = "%s(%s, %s)" % (rng.choice(["add", "sub", "mul", "protectedDiv"]),
                          left, right)
    if rng.random() < 0.3:
        out = "%s(%s)" % (rng.choice(["sin", "cos", "neg"]), out)
    return out


def main():
    pset = mg.arith_pset(10, False)
    dpset = configs.pset_for("symreg10")
    fl = Flattener(dpset)

    def slots(s):
        return int(fl.flatten_py([dgp.PrimitiveTree.from_string(s, dpset)])
                   .depth[0])

    random.seed(500)                      # gp.genFull draws from `random`
    rng = random.Random(9)
    trees = []
    for s in PLAN:
        while True:                       # constant folds can lower the need
            t = skeleton(pset, rng, s - 1)
            if "sin(" not in t and "cos(" not in t:
                t = "sin(%s)" % t
            if slots(t) == s:
                break
        trees.append(t)
    while len(trees) < len(PLAN) + N_REDO:   # the redo path (glibc sin/cos)
        base = skeleton(pset, rng, 5)
        a, b, c, d, e = (rng.randrange(10) for _ in range(5))
        hot = ("sin(protectedDiv(protectedDiv(ARG%d, sub(ARG%d, ARG%d)), "
               "sub(ARG%d, ARG%d)))" % (a, b, c, d, e))
        t = "%s(%s, %s)" % (rng.choice(["add", "mul", "sub"]), base, hot)
        if 6 <= slots(t) <= 12:
            trees.append(t)
    got = [slots(t) for t in trees]
    assert all(6 <= v <= 12 for v in got), sorted(set(got))
    print("slots:", {v: got.count(v) for v in sorted(set(got))},
          "nodes:", sum(len(dgp.PrimitiveTree.from_string(t, dpset))
                        for t in trees), flush=True)
    X, Y = datasets.symreg10_cases(N_CASES, SEED)
    mg.symreg_fixture("c4_deep_core", pset, trees, X, Y,
                      {"pset": "symreg10",
                       "data": {"kind": "symreg10_cases", "n": N_CASES,
                                "seed": SEED}})


if __name__ == "__main__":
    main()
