#!/usr/bin/env python3
"""Evolved C4 populations for bench.py's ``evolved`` leg (and its tests).

The headline population is generation 0 (``genHalfAndHalf(4, 8)``); a GP
run's later generations are larger and deeper (``staticLimit(17)``).  (They
are also sin/cos-heavier — 20 % of the nodes against 14 % — and, despite
heights up to 17, need at most 4 operand-stack slots: bloat grows chains,
not balanced trees, so the D = 5 core runs all of them and the deep core
stays for rare balanced shapes, tests/golden/c4_deep_core.)  This script
runs the
reference's symbolic-regression loop (``examples/gp/symbreg.py:47-90``:
``genHalfAndHalf(1, 2)`` start, tournament 3, ``cxOnePoint``,
``mutUniform(genFull(0, 2))``, both decorated with
``staticLimit(height, 17)``, ``eaSimple(cxpb=0.5, mutpb=0.1)``) on the C4
primitive set and target (``unwrapped_ball`` over 10 variables), with the
fitness computed on 512 cases by numpy (a generation-only stand-in with the
same primitive names; the trees, not these fitnesses, are the output).
Several seeded runs; the final populations go to
``tests/golden/c4_evolved.json.gz`` as tree strings.

Usage: python scripts/evolve_c4.py [runs=8] [pop=512] [gens=150]
"""
import gzip
import json
import operator
import os
import random
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from deap_amd import algorithms, base, configs, creator, datasets, gp, tools  # noqa: E402


def _pdiv(a, b):
    with np.errstate(all="ignore"):
        return np.where(b == 0, 1.0, a / np.where(b == 0, 1.0, b))


def numpy_twin():
    """The C4 primitive set with numpy bodies under the same names (tree
    strings parse in configs.pset_for("symreg10"))."""
    pset = gp.PrimitiveSet("MAIN", 10)
    pset.addPrimitive(np.add, 2, name="add")
    pset.addPrimitive(np.subtract, 2, name="sub")
    pset.addPrimitive(np.multiply, 2, name="mul")
    pset.addPrimitive(_pdiv, 2, name="protectedDiv")
    pset.addPrimitive(np.negative, 1, name="neg")
    pset.addPrimitive(np.cos, 1, name="cos")
    pset.addPrimitive(np.sin, 1, name="sin")
    pset.addEphemeralConstant("rand101", configs.rand101)
    return pset


def run(seed, pop_n, gens, X, y):
    pset = numpy_twin()
    if not hasattr(creator, "EvoFit"):
        creator.create("EvoFit", base.Fitness, weights=(-1.0,))
        creator.create("EvoInd", gp.PrimitiveTree, fitness=creator.EvoFit)
    tb = base.Toolbox()
    tb.register("expr", gp.genHalfAndHalf, pset=pset, min_=1, max_=2)
    tb.register("individual", tools.initIterate, creator.EvoInd, tb.expr)
    tb.register("population", tools.initRepeat, list, tb.individual)
    cols = [X[i] for i in range(X.shape[0])]

    def evaluate(ind):
        f = gp.compile(ind, pset)
        with np.errstate(all="ignore"):
            v = np.broadcast_to(np.asarray(f(*cols), dtype=np.float64), y.shape)
            mse = float(np.mean((v - y) ** 2))
        return (mse if np.isfinite(mse) else 1e300,)
    tb.register("evaluate", evaluate)
    tb.register("select", tools.selTournament, tournsize=3)
    tb.register("mate", gp.cxOnePoint)
    tb.register("expr_mut", gp.genFull, min_=0, max_=2)
    tb.register("mutate", gp.mutUniform, expr=tb.expr_mut, pset=pset)
    tb.decorate("mate", gp.staticLimit(key=operator.attrgetter("height"), max_value=17))
    tb.decorate("mutate", gp.staticLimit(key=operator.attrgetter("height"), max_value=17))
    random.seed(seed)
    pop = tb.population(n=pop_n)
    pop, _ = algorithms.eaSimple(pop, tb, 0.5, 0.1, gens, verbose=False)
    return [str(t) for t in pop]


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    pop_n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    gens = int(sys.argv[3]) if len(sys.argv) > 3 else 150
    X, Y = datasets.symreg10_cases(512, 31)
    y = Y[0]
    trees = []
    for r in range(runs):
        got = run(1000 + r, pop_n, gens, X, y)
        trees += got
        lens = [len(gp.PrimitiveTree.from_string(t, configs.pset_for("symreg10")))
                for t in got]
        print("run %d: %d trees, mean length %.1f, max %d" % (r, len(got),
              sum(lens) / len(lens), max(lens)), flush=True)
    out = os.path.join(REPO, "tests", "golden", "c4_evolved.json.gz")
    with gzip.open(out, "wt") as fh:
        json.dump({"pset": "symreg10", "trees": trees,
                   "source": "scripts/evolve_c4.py %d %d %d" % (runs, pop_n, gens)}, fh)
    print("wrote", out, len(trees), "trees")


if __name__ == "__main__":
    main()
