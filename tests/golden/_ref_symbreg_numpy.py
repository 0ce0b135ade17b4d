"""Evaluate trees with the reference's examples/gp/symbreg_numpy.py and run
its seed-318 evolution; print the results as JSON.  Executed by
make_golden.py with PYTHONPATH pointing at the 2to3 scratch copy of the
reference; build container only.

Output: ``{"trees": [...], "fitness": [hex], "logbook": {...}}``.  Trees are
drawn by the reference's own ``gp.genHalfAndHalf`` on the example's pset, plus
hand-written edge cases (division by zero/inf/nan, overflow to inf, sin/cos of
inf -> nan, constant-only trees)."""
import json
import os
import random
import sys
import warnings

copy = os.environ["PYTHONPATH"].split(os.pathsep)[0]
sys.path.insert(0, os.path.join(copy, "examples", "gp"))
import numpy  # noqa: E402
import symbreg_numpy as ex  # noqa: E402  (reference example)
from deap import algorithms, gp, tools  # noqa: E402

warnings.simplefilter("ignore")


def h(v):
    return float(v).hex()


def gen(seed, n, lo, hi):
    random.seed(seed)
    return [str(gp.PrimitiveTree(gp.genHalfAndHalf(ex.pset, min_=lo,
                                                    max_=hi)))
            for _ in range(n)]


def nest(fmt, inner, times):
    s = inner
    for _ in range(times):
        s = fmt.format(s)
    return s


big = nest("vmul({0}, {0})", "vmul(x, 1000)", 6)          # d**2 -> inf
huge = nest("vmul({0}, {0})", "vmul(x, 1000)", 7)         # inf for |x|>.26
two = nest("vmul({0}, {0})", "vadd(1, 1)", 6)             # int64 2**64 wraps
edge = [
    "protectedDiv(x, vsub(x, x))", "protectedDiv(1, 0)", "protectedDiv(0, 0)",
    "protectedDiv(vsub(x, x), vsub(x, x))", "vcos(protectedDiv(1, 0))",
    "vsin(vneg(1))", "protectedDiv(1, x)", "protectedDiv(x, x)",
    "vcos(x)", "vsin(x)", "vneg(x)", "x", "1", "0", "-1",
    big, "vsin(%s)" % big, "vcos(%s)" % big, "vsub(%s, %s)" % (big, big),
    "protectedDiv(%s, %s)" % (big, big), "protectedDiv(x, %s)" % big,
    "vmul(%s, 0)" % big, "vadd(%s, vneg(%s))" % (big, big),
    "protectedDiv(1, %s)" % big, two, "vadd(%s, x)" % two,
    "protectedDiv(%s, 0)" % big, huge, "vsin(%s)" % huge,
    "vcos(%s)" % huge, "vsub(%s, %s)" % (huge, huge),
    "protectedDiv(%s, %s)" % (huge, huge), "protectedDiv(x, %s)" % huge,
    "vmul(%s, 0)" % huge, "protectedDiv(vsin(%s), 0)" % huge,
    "vmul(vsin(x), protectedDiv(1, vsub(%s, %s)))" % (huge, huge),
    nest("vsin({0})", "x", 30), nest("vcos({0})", "vmul(x, 50)", 5),
    "protectedDiv(vcos(x), vsin(vsub(x, x)))",
]
trees = gen(601, 1000, 1, 2) + gen(602, 1000, 2, 6) + edge
fits = []
for s in trees:
    with numpy.errstate(all="ignore"):
        fits.append(h(ex.evalSymbReg(s)[0]))

# the example's main() (symbreg_numpy.py:76-90) with the logbook kept
random.seed(318)
pop = ex.toolbox.population(n=300)
hof = tools.HallOfFame(1)
stats = tools.Statistics(lambda ind: ind.fitness.values)
stats.register("avg", numpy.mean)
stats.register("std", numpy.std)
stats.register("min", numpy.min)
stats.register("max", numpy.max)
with numpy.errstate(all="ignore"):
    pop, log = algorithms.eaSimple(pop, ex.toolbox, 0.5, 0.1, 40, stats,
                                   halloffame=hof, verbose=False)
book = {"gen": log.select("gen"), "nevals": log.select("nevals")}
for f in ("avg", "std", "min", "max"):
    book[f] = [h(v) for v in log.select(f)]
book["hof"] = str(hof[0])
book["hof_fitness"] = h(hof[0].fitness.values[0])
print(json.dumps({"trees": trees, "fitness": fits, "n_edge": len(edge),
                  "logbook": book}))
