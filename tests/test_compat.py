"""The DEAP-API surface the GP path needs (deap_amd.{base,creator,gp,tools,
algorithms}) behaves like the reference: seeded runs consume ``random``
exactly like it, so the reference's own config-1 run is reproduced."""
import copy
import math
import operator
import pickle
import random

import numpy as np
import pytest

from conftest import load_golden
from deap_amd import algorithms, base, configs, creator, gp, tools


def test_c1_cpu_path_reproduces_reference_logbook_exactly():
    """examples/gp/symbreg.py main() with the CPU evaluate (gp.compile + per
    case loop + fsum) must match the reference's recorded run bit for bit."""
    g = load_golden("c1_logbook")
    pset = configs.pset_for("symbreg")
    creator.create("FitnessMinC", base.Fitness, weights=(-1.0,))
    creator.create("IndividualC", gp.PrimitiveTree,
                   fitness=creator.FitnessMinC)
    tb = base.Toolbox()
    tb.register("expr", gp.genHalfAndHalf, pset=pset, min_=1, max_=2)
    tb.register("individual", tools.initIterate, creator.IndividualC, tb.expr)
    tb.register("population", tools.initRepeat, list, tb.individual)
    tb.register("compile", gp.compile, pset=pset)

    def evalSymbReg(individual, points):
        func = tb.compile(expr=individual)
        sq = ((func(x) - x**4 - x**3 - x**2 - x)**2 for x in points)
        return math.fsum(sq) / len(points),
    tb.register("evaluate", evalSymbReg, points=[x / 10. for x in
                                                 range(-10, 10)])
    tb.register("select", tools.selTournament, tournsize=3)
    tb.register("mate", gp.cxOnePoint)
    tb.register("expr_mut", gp.genFull, min_=0, max_=2)
    tb.register("mutate", gp.mutUniform, expr=tb.expr_mut, pset=pset)
    tb.decorate("mate", gp.staticLimit(key=operator.attrgetter("height"),
                                       max_value=17))
    tb.decorate("mutate", gp.staticLimit(key=operator.attrgetter("height"),
                                         max_value=17))
    random.seed(318)
    pop = tb.population(n=300)
    hof = tools.HallOfFame(1)
    ms = tools.MultiStatistics(
        fitness=tools.Statistics(lambda ind: ind.fitness.values),
        size=tools.Statistics(len))
    for nm, fn in (("avg", np.mean), ("std", np.std), ("min", np.min),
                   ("max", np.max)):
        ms.register(nm, fn)
    pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.1, 40, stats=ms,
                                   halloffame=hof, verbose=False)
    assert log.select("gen") == g["gen"]
    assert log.select("nevals") == g["nevals"]
    for chap in ("fitness", "size"):
        for f in ("avg", "std", "min", "max"):
            got = [float(v).hex() for v in log.chapters[chap].select(f)]
            assert got == g["%s_%s" % (chap, f)], (chap, f)
    assert str(hof[0]) == g["hof"]
    assert hof[0].fitness.values[0].hex() == g["hof_fitness"]
    assert "fitness" in str(log).splitlines()[0]


def numpy_example_run(evaluate, tag):
    """examples/gp/symbreg_numpy.py main() (seed 318, pop 300, 40 gens, no
    height limit) with *evaluate* registered; returns (logbook, hof)."""
    pset = configs.pset_for("symbreg_numpy")
    creator.create("FitnessMin" + tag, base.Fitness, weights=(-1.0,))
    creator.create("Individual" + tag, gp.PrimitiveTree,
                   fitness=getattr(creator, "FitnessMin" + tag))
    tb = base.Toolbox()
    tb.register("expr", gp.genHalfAndHalf, pset=pset, min_=1, max_=2)
    tb.register("individual", tools.initIterate,
                getattr(creator, "Individual" + tag), tb.expr)
    tb.register("population", tools.initRepeat, list, tb.individual)
    tb.register("select", tools.selTournament, tournsize=3)
    tb.register("mate", gp.cxOnePoint)
    tb.register("expr_mut", gp.genFull, min_=0, max_=2)
    tb.register("mutate", gp.mutUniform, expr=tb.expr_mut, pset=pset)
    evaluate(tb, pset)
    random.seed(318)
    pop = tb.population(n=300)
    hof = tools.HallOfFame(1)
    stats = tools.Statistics(lambda ind: ind.fitness.values)
    for nm, fn in (("avg", np.mean), ("std", np.std), ("min", np.min),
                   ("max", np.max)):
        stats.register(nm, fn)
    with np.errstate(all="ignore"):
        pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.1, 40, stats,
                                       halloffame=hof, verbose=False)
    return log, hof


def same_float(a, b, rel=0.0):
    a, b = float(a), float(b)
    if math.isnan(b):
        return math.isnan(a)
    return a == b or abs(a - b) <= rel * abs(b)


def test_numpy_example_cpu_path_reproduces_reference_logbook():
    """symbreg_numpy.py with its own vectorised evaluate on this API."""
    from deap_amd import datasets
    g = load_golden("np_symbreg")["logbook"]
    X, V = datasets.symbreg_numpy_points()

    def register(tb, pset):
        def evalSymbReg(individual):
            func = gp.compile(individual, pset)
            return np.sum((func(X[0]) - V[0]) ** 2),
        tb.register("evaluate", evalSymbReg)
    log, hof = numpy_example_run(register, "NpC")
    assert log.select("nevals") == g["nevals"]
    for f in ("avg", "std", "min", "max"):
        got = [float(v).hex() for v in log.select(f)]
        assert got == g[f], f
    assert str(hof[0]) == g["hof"]


def adf_example_run(register, tag, batch_map=False):
    """examples/gp/adf_symbreg.py main() (seed 1024, pop 100, 40 gens, its
    own generational loop) with *register(tb, psets)* installing evaluate;
    returns (logbook, hof)."""
    psets = configs.pset_for("adf_symbreg")
    main_set, adf0, adf1, adf2 = psets
    creator.create("FitnessMin" + tag, base.Fitness, weights=(-1.0,))
    creator.create("Tree" + tag, gp.PrimitiveTree)
    creator.create("Individual" + tag, list,
                   fitness=getattr(creator, "FitnessMin" + tag))
    Tree, Ind = getattr(creator, "Tree" + tag), \
        getattr(creator, "Individual" + tag)
    tb = base.Toolbox()
    tb.register("adf_expr0", gp.genFull, pset=adf0, min_=1, max_=2)
    tb.register("adf_expr1", gp.genFull, pset=adf1, min_=1, max_=2)
    tb.register("adf_expr2", gp.genFull, pset=adf2, min_=1, max_=2)
    tb.register("main_expr", gp.genHalfAndHalf, pset=main_set, min_=1,
                max_=2)
    tb.register("ADF0", tools.initIterate, Tree, tb.adf_expr0)
    tb.register("ADF1", tools.initIterate, Tree, tb.adf_expr1)
    tb.register("ADF2", tools.initIterate, Tree, tb.adf_expr2)
    tb.register("MAIN", tools.initIterate, Tree, tb.main_expr)
    tb.register("individual", tools.initCycle, Ind,
                [tb.MAIN, tb.ADF0, tb.ADF1, tb.ADF2])
    tb.register("population", tools.initRepeat, list, tb.individual)
    tb.register("select", tools.selTournament, tournsize=3)
    tb.register("mate", gp.cxOnePoint)
    tb.register("expr", gp.genFull, min_=1, max_=2)
    tb.register("mutate", gp.mutUniform, expr=tb.expr)
    register(tb, psets)
    stats = tools.Statistics(lambda ind: ind.fitness.values)
    for nm, fn in (("avg", np.mean), ("std", np.std), ("min", np.min),
                   ("max", np.max)):
        stats.register(nm, fn)

    def evaluate_all(inds):
        for ind, fit in zip(inds, tb.map(tb.evaluate, inds)):
            ind.fitness.values = fit
    random.seed(1024)
    tb.individual()
    pop = tb.population(n=100)
    hof = tools.HallOfFame(1)
    log = tools.Logbook()
    evaluate_all(pop)
    hof.update(pop)
    log.record(gen=0, evals=len(pop), **stats.compile(pop))
    for g in range(1, 40):
        off = [tb.clone(ind) for ind in tb.select(pop, len(pop))]
        for i1, i2 in zip(off[::2], off[1::2]):
            for t1, t2 in zip(i1, i2):
                if random.random() < 0.5:
                    tb.mate(t1, t2)
                    del i1.fitness.values
                    del i2.fitness.values
        for ind in off:
            for tree, pset in zip(ind, psets):
                if random.random() < 0.2:
                    tb.mutate(individual=tree, pset=pset)
                    del ind.fitness.values
        invalids = [ind for ind in off if not ind.fitness.valid]
        evaluate_all(invalids)
        pop = off
        hof.update(pop)
        log.record(gen=g, evals=len(invalids), **stats.compile(pop))
    return log, hof


def test_adf_example_cpu_path_reproduces_reference_logbook():
    """adf_symbreg.py with gp.compileADF + builtin-sum evaluate on this API
    must match the reference's recorded run bit for bit."""
    g = load_golden("adf_symbreg")["logbook"]

    def register(tb, psets):
        def evalSymbReg(individual):
            func = gp.compileADF(individual, psets)
            values = (x / 10. for x in range(-10, 10))
            return sum((func(x) - (x**4 + x**3 + x**2 + x))**2
                       for x in values),
        tb.register("evaluate", evalSymbReg)
    log, hof = adf_example_run(register, "AdfC")
    assert log.select("evals") == g["evals"]
    for f in ("avg", "std", "min", "max"):
        assert [float(v).hex() for v in log.select(f)] == g[f], f
    assert [str(t) for t in hof[0]] == g["hof"]


def test_tree_string_roundtrip_and_height():
    for name, gen, lo, hi in (("symbreg", "half", 1, 6),
                              ("mux11", "full", 2, 4),
                              ("spambase", "half", 2, 6)):
        pset = configs.pset_for(name)
        for t in configs.population(pset, gen, 200, 3, lo, hi):
            s = str(t)
            back = gp.PrimitiveTree.from_string(s, pset)
            assert str(back) == s
            assert back.height == t.height
            assert len(back) == len(t)


def test_search_subtree_and_setitem_checks():
    pset = configs.pset_for("symbreg")
    t = gp.PrimitiveTree.from_string("add(mul(x, 1), neg(x))", pset)
    assert t.searchSubtree(1) == slice(1, 4)
    assert t.searchSubtree(4) == slice(4, 6)
    with pytest.raises(ValueError):
        t[0] = t[5]              # arity mismatch
    with pytest.raises(ValueError):
        t[1:4] = [t[0]]          # incomplete subtree


def test_typed_generation_respects_types():
    pset = configs.pset_for("spambase")
    for t in configs.population(pset, "half", 300, 11, 2, 6):
        need = [bool]
        for node in t:
            want = need.pop()
            assert issubclass(node.ret, want)
            need.extend(reversed(getattr(node, "args", [])))


def test_pickle_individual_roundtrip():
    creator.create("FitnessMaxP", base.Fitness, weights=(1.0,))
    creator.create("IndividualP", gp.PrimitiveTree,
                   fitness=creator.FitnessMaxP)
    pset = configs.pset_for("symbreg")
    random.seed(1)
    ind = creator.IndividualP(gp.genFull(pset, 2, 3))
    ind.fitness.values = (1.5,)
    back = pickle.loads(pickle.dumps(ind, pickle.HIGHEST_PROTOCOL))
    assert str(back) == str(ind)
    assert back.fitness == ind.fitness


def test_toolbox_partial_and_clone():
    tb = base.Toolbox()
    tb.register("f", lambda a, b=2: a + b, b=5)
    assert tb.f(1) == 6 and tb.f.__name__ == "f"
    creator.create("FitnessMinT", base.Fitness, weights=(-1.0,))
    creator.create("IndT", gp.PrimitiveTree, fitness=creator.FitnessMinT)
    pset = configs.pset_for("symbreg")
    random.seed(2)
    a = creator.IndT(gp.genFull(pset, 1, 2))
    a.fitness.values = (3.0,)
    b = tb.clone(a)
    assert b == a and b is not a and b.fitness is not a.fitness
    del b.fitness.values
    assert a.fitness.valid and not b.fitness.valid
    c = copy.deepcopy(a)
    assert c[0] is a[0]          # nodes are shared, like the reference


def test_halloffame_and_selection():
    creator.create("FitnessMaxH", base.Fitness, weights=(1.0,))

    class Ind(list):
        def __init__(self, v):
            super().__init__([v])
            self.fitness = creator.FitnessMaxH((v,))
    pop = [Ind(v) for v in (3, 1, 4, 1, 5, 9, 2, 6)]
    hof = tools.HallOfFame(3)
    hof.update(pop)
    assert [i[0] for i in hof] == [9, 6, 5]
    random.seed(0)
    sel = tools.selTournament(pop, 8, tournsize=3)
    assert len(sel) == 8 and all(s in pop for s in sel)


def test_ea_generate_update_asks_and_tells():
    pset = configs.pset_for("symbreg")
    creator.create("FitnessMinGU", base.Fitness, weights=(-1.0,))
    creator.create("IndividualGU", gp.PrimitiveTree,
                   fitness=creator.FitnessMinGU)
    tb = base.Toolbox()
    tb.register("individual", tools.initIterate, creator.IndividualGU,
                lambda: gp.genHalfAndHalf(pset, 1, 3))
    tb.register("generate", tools.initRepeat, list, tb.individual, 30)
    told = []
    tb.register("update", lambda pop: told.append(len(pop)))
    tb.register("evaluate", lambda ind: (float(len(ind)),))
    random.seed(3)
    pop, log = algorithms.eaGenerateUpdate(tb, 5, verbose=False)
    assert told == [30] * 5 and log.select("nevals") == [30] * 5
    assert log.select("gen") == list(range(5))
    assert all(ind.fitness.values == (float(len(ind)),) for ind in pop)
