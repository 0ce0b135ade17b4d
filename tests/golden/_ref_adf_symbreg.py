"""Evaluate ADF individuals with the reference's examples/gp/adf_symbreg.py
and run its seed-1024 evolution; print the results as JSON.  Executed by
make_golden.py with PYTHONPATH pointing at the 2to3 scratch copy of the
reference; build container only.

Output: ``{"individuals": [[main, adf0, adf1, adf2], ...], "fitness": [...],
"error": [...], "logbook": {...}}``.  Individuals come from the example's
own ``toolbox.population`` (seeded), plus hand-written ones: ADF arguments
the body never reads (evaluated anyway by the eager call, and raising),
nested ADF calls, constant-only arguments, overflow of ``d**2``."""
import json
import os
import random
import sys

copy = os.environ["PYTHONPATH"].split(os.pathsep)[0]
sys.path.insert(0, os.path.join(copy, "examples", "gp"))
import numpy  # noqa: E402
import adf_symbreg as ex  # noqa: E402  (reference example)
from deap import gp, tools  # noqa: E402


def h(v):
    return float(v).hex()


def run(ind):
    try:
        return h(ex.evalSymbReg(ind)[0]), None
    except (ValueError, OverflowError, ZeroDivisionError, SyntaxError,
            TypeError, MemoryError, RecursionError) as exc:
        return None, type(exc).__name__


def nest(fmt, inner, times):
    s = inner
    for _ in range(times):
        s = fmt.format(s)
    return s


def from_strings(strs):
    return ex.creator.Individual(
        [ex.creator.Tree(gp.PrimitiveTree.from_string(s, p))
         for s, p in zip(strs, ex.psets)])


inds = []
for seed in (1101, 1102):
    random.seed(seed)
    inds += [[str(t) for t in ind] for ind in ex.toolbox.population(n=500)]

inv = "protectedDiv(1, x)"
big = nest("mul({0}, {0})", inv, 9)        # inf at |x| <= 0.2 (x != 0)
big8 = nest("mul({0}, {0})", inv, 8)       # finite; its square overflows
simple = ["add(ARG0, ARG1)", "ARG0", "ARG1"]
edge = [
    ["ADF0(x, x)"] + simple,
    ["ADF2(x, cos(%s))" % big, "ARG0", "ARG0", "ARG0"],     # dead arg raises
    ["ADF2(cos(%s), x)" % big, "ARG0", "ARG0", "ARG1"],     # dead arg raises
    ["ADF2(x, %s)" % big, "ARG0", "ARG0", "ARG0"],          # dead, inf only
    ["ADF1(%s, x)" % big8, "ARG0", "ARG0", "ARG1"],         # d**2 overflow
    ["ADF0(x, add(x, 1))", "mul(ARG0, add(ARG0, ARG1))", "ARG0", "ARG1"],
    ["ADF0(x, neg(x))", "ADF1(ARG0, ADF2(ARG1, ARG0))",
     "sub(ADF2(ARG0, ARG1), ARG1)", "protectedDiv(ARG0, ARG1)"],
    ["ADF0(1, -1)", "add(ARG0, ARG1)", "ARG0", "ARG1"],
    ["ADF1(0, 0)", "ARG0", "protectedDiv(ARG0, ARG1)", "ARG1"],
    ["add(ADF0(x, x), ADF2(x, 1))", "sin(ARG0)", "cos(ARG1)",
     "mul(ARG0, ARG1)"],
    ["x", "ARG0", "ARG0", "ARG0"],
    ["ADF2(ADF2(x, x), ADF2(x, ADF2(x, x)))", "ARG0", "ARG0",
     "mul(ARG0, ARG1)"],
]
inds += edge
fits, errs = [], []
for strs in inds:
    f, e = run(from_strings(strs))
    fits.append(f)
    errs.append(e)

# the example's main() (adf_symbreg.py:129-179) with the logbook kept
random.seed(1024)
ind = ex.toolbox.individual()
pop = ex.toolbox.population(n=100)
hof = tools.HallOfFame(1)
stats = tools.Statistics(lambda ind: ind.fitness.values)
stats.register("avg", numpy.mean)
stats.register("std", numpy.std)
stats.register("min", numpy.min)
stats.register("max", numpy.max)
logbook = tools.Logbook()
for ind in pop:
    ind.fitness.values = ex.toolbox.evaluate(ind)
hof.update(pop)
logbook.record(gen=0, evals=len(pop), **stats.compile(pop))
for g in range(1, 40):
    offspring = ex.toolbox.select(pop, len(pop))
    offspring = [ex.toolbox.clone(ind) for ind in offspring]
    for ind1, ind2 in zip(offspring[::2], offspring[1::2]):
        for tree1, tree2 in zip(ind1, ind2):
            if random.random() < 0.5:
                ex.toolbox.mate(tree1, tree2)
                del ind1.fitness.values
                del ind2.fitness.values
    for ind in offspring:
        for tree, pset in zip(ind, ex.psets):
            if random.random() < 0.2:
                ex.toolbox.mutate(individual=tree, pset=pset)
                del ind.fitness.values
    invalids = [ind for ind in offspring if not ind.fitness.valid]
    for ind in invalids:
        ind.fitness.values = ex.toolbox.evaluate(ind)
    pop = offspring
    hof.update(pop)
    logbook.record(gen=g, evals=len(invalids), **stats.compile(pop))
book = {"gen": logbook.select("gen"), "evals": logbook.select("evals")}
for f in ("avg", "std", "min", "max"):
    book[f] = [h(v) for v in logbook.select(f)]
book["hof"] = [str(t) for t in hof[0]]
book["hof_fitness"] = h(hof[0].fitness.values[0])
print(json.dumps({"individuals": inds, "fitness": fits, "error": errs,
                  "n_edge": len(edge), "logbook": book}))
