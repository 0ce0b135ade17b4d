"""The five BASELINE configurations, built on the DEAP-API surface.

Each builder mirrors the reference example it cites (primitive set, fitness
formula, population generator) and returns a :class:`Config`.

C1  examples/gp/symbreg.py      quartic symbolic regression, 20 points
C2  examples/gp/multiplexer.py  11-multiplexer, 2048 boolean cases
C3  examples/gp/parity.py       even-6 parity, 64 cases
C4  synthetic 10-variable regression (symbreg primitives, 10 arguments,
    target deap/benchmarks/gp.py:60-72 unwrapped_ball), 2**20 cases
C5  examples/gp/spambase.py     strongly typed GP on spambase-like rows
NP  examples/gp/symbreg_numpy.py vectorised quartic regression (numpy
    ufunc primitives, inf/nan-to-1 protectedDiv, numpy.sum SSE)
ADF examples/gp/adf_symbreg.py  quartic regression with three ADFs
    (individual = [main, ADF0, ADF1, ADF2], builtin-sum SSE)
"""
import itertools
import math
import operator
import random
from collections import namedtuple

import numpy

from . import datasets, gp
from .evaluator import (BooleanHits, SymbRegMSE, SymbRegNumpySSE,
                        SymbRegSumSSE, TypedBoolHits)

Config = namedtuple("Config", "name pset spec generate weights")


def protectedDiv(left, right):
    """examples/gp/symbreg.py:29-33."""
    try:
        return left / right
    except ZeroDivisionError:
        return 1


def np_protectedDiv(left, right):
    """examples/gp/symbreg_numpy.py:28-36 (inf/nan quotients become 1)."""
    with numpy.errstate(divide="ignore", invalid="ignore"):
        x = numpy.divide(left, right)
        if isinstance(x, numpy.ndarray):
            x[~numpy.isfinite(x)] = 1
        elif not numpy.isfinite(x):
            x = 1
    return x


def if_then_else(condition, out1, out2):
    """examples/gp/multiplexer.py:27-28."""
    return out1 if condition else out2


def rand101():
    """examples/gp/symbreg.py:43."""
    return random.randint(-1, 1)


def rand100():
    """examples/gp/spambase.py:67."""
    return random.random() * 100


def arith_pset(n_args, rename_x=False, trig=True):
    """symbreg.py:35-44 primitive set (with *n_args* arguments)."""
    pset = gp.PrimitiveSet("MAIN", n_args)
    pset.addPrimitive(operator.add, 2)
    pset.addPrimitive(operator.sub, 2)
    pset.addPrimitive(operator.mul, 2)
    pset.addPrimitive(protectedDiv, 2)
    pset.addPrimitive(operator.neg, 1)
    if trig:
        pset.addPrimitive(math.cos, 1)
        pset.addPrimitive(math.sin, 1)
    pset.addEphemeralConstant("rand101", rand101)
    if rename_x:
        pset.renameArguments(ARG0="x")
    return pset


def numpy_pset():
    """symbreg_numpy.py:38-46."""
    pset = gp.PrimitiveSet("MAIN", 1)
    pset.addPrimitive(numpy.add, 2, name="vadd")
    pset.addPrimitive(numpy.subtract, 2, name="vsub")
    pset.addPrimitive(numpy.multiply, 2, name="vmul")
    pset.addPrimitive(np_protectedDiv, 2, name="protectedDiv")
    pset.addPrimitive(numpy.negative, 1, name="vneg")
    pset.addPrimitive(numpy.cos, 1, name="vcos")
    pset.addPrimitive(numpy.sin, 1, name="vsin")
    pset.addEphemeralConstant("rand101", rand101)
    pset.renameArguments(ARG0="x")
    return pset


def _arith(name, n_args):
    pset = gp.PrimitiveSet(name, n_args)
    pset.addPrimitive(operator.add, 2)
    pset.addPrimitive(operator.sub, 2)
    pset.addPrimitive(operator.mul, 2)
    pset.addPrimitive(protectedDiv, 2)
    pset.addPrimitive(operator.neg, 1)
    pset.addPrimitive(math.cos, 1)
    pset.addPrimitive(math.sin, 1)
    return pset


def adf_psets():
    """adf_symbreg.py:35-80: ``(MAIN, ADF0, ADF1, ADF2)`` — compileADF's
    ``psets``; ADF0 calls ADF1/ADF2, ADF1 calls ADF2, MAIN calls all."""
    adf2 = _arith("ADF2", 2)
    adf1 = _arith("ADF1", 2)
    adf1.addADF(adf2)
    adf0 = _arith("ADF0", 2)
    adf0.addADF(adf1)
    adf0.addADF(adf2)
    main = _arith("MAIN", 1)
    main.addEphemeralConstant("rand101", rand101)
    main.addADF(adf0)
    main.addADF(adf1)
    main.addADF(adf2)
    main.renameArguments(ARG0="x")
    return (main, adf0, adf1, adf2)


def mux_pset():
    """multiplexer.py:56-62."""
    pset = gp.PrimitiveSet("MAIN", 11, "IN")
    pset.addPrimitive(operator.and_, 2)
    pset.addPrimitive(operator.or_, 2)
    pset.addPrimitive(operator.not_, 1)
    pset.addPrimitive(if_then_else, 3)
    pset.addTerminal(1)
    pset.addTerminal(0)
    return pset


def parity_pset():
    """parity.py:49-55."""
    pset = gp.PrimitiveSet("MAIN", 6, "IN")
    pset.addPrimitive(operator.and_, 2)
    pset.addPrimitive(operator.or_, 2)
    pset.addPrimitive(operator.xor, 2)
    pset.addPrimitive(operator.not_, 1)
    pset.addTerminal(1)
    pset.addTerminal(0)
    return pset


def spam_pset():
    """spambase.py:38-69."""
    pset = gp.PrimitiveSetTyped("MAIN", itertools.repeat(float, 57), bool,
                                "IN")
    pset.addPrimitive(operator.and_, [bool, bool], bool)
    pset.addPrimitive(operator.or_, [bool, bool], bool)
    pset.addPrimitive(operator.not_, [bool], bool)
    pset.addPrimitive(operator.add, [float, float], float)
    pset.addPrimitive(operator.sub, [float, float], float)
    pset.addPrimitive(operator.mul, [float, float], float)
    pset.addPrimitive(protectedDiv, [float, float], float)
    pset.addPrimitive(operator.lt, [float, float], bool)
    pset.addPrimitive(operator.eq, [float, float], bool)
    pset.addPrimitive(if_then_else, [bool, float, float], float)
    pset.addEphemeralConstant("rand100", rand100, float)
    pset.addTerminal(False, bool)
    pset.addTerminal(True, bool)
    return pset


_PSETS = {}


def pset_for(name):
    """Primitive sets are cached: ephemeral classes are module-global, as in
    the reference (gp.py:393-397)."""
    if name not in _PSETS:
        _PSETS[name] = {
            "symbreg": lambda: arith_pset(1, rename_x=True),
            "symreg10": lambda: arith_pset(10),
            "symreg10_notrig": lambda: arith_pset(10, trig=False),
            "mux11": mux_pset,
            "parity6": parity_pset,
            "spambase": spam_pset,
            "symbreg_numpy": numpy_pset,
            "adf_symbreg": adf_psets,
        }[name]()
    return _PSETS[name]


def _golden_file(name):
    """A data file committed with the test fixtures (tests/golden)."""
    import os
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), "tests", "golden", name)


def spec_for(name, data=None):
    """Fitness spec of a golden/bench data description."""
    data = data or {}
    kind = data.get("kind")
    if name == "symbreg":
        return SymbRegMSE.quartic()
    if name == "symreg10":
        X, y = datasets.symreg10_cases(data.get("n", 2 ** 20),
                                       data.get("seed", 2024))
        return SymbRegMSE(X, y)
    if name == "mux11":
        ins, outs = datasets.mux11_table()
        return BooleanHits(ins, outs)
    if name == "parity6":
        ins, outs = datasets.parity6_table()
        return BooleanHits(ins, outs)
    if name == "spambase":
        if kind == "spambase_csv":      # the reference's own rows
            X, lab = datasets.spambase_csv(data.get("path") or _golden_file(
                data.get("file", "spambase.csv.gz")))
        else:
            X, lab = datasets.spambase_like(data.get("n", 4601),
                                            data.get("seed", 1234))
        return TypedBoolHits(X, lab)
    if name == "symbreg_numpy":
        return SymbRegNumpySSE.linspace(data.get("n", 10000))
    if name == "adf_symbreg":
        return SymbRegSumSSE.adf_quartic()
    raise KeyError((name, kind))


def population(pset, generator, n, seed, min_, max_):
    """Seeded population of PrimitiveTrees from a reference generator."""
    random.seed(seed)
    gen = {"full": gp.genFull, "grow": gp.genGrow,
           "half": gp.genHalfAndHalf}[generator]
    return [gp.PrimitiveTree(gen(pset, min_, max_)) for _ in range(n)]


def headline_c4(pop=65536, cases=2 ** 20, seed=2024, min_=4, max_=8,
                trig=True):
    """bench.py's workload (config 4): ``(pset, population, X[10, cases],
    y[1, cases])`` — ``genHalfAndHalf(min_, max_)`` trees seeded with
    ``seed``, X ~ U(-1, 1) from ``default_rng(seed)``, y the reference's
    ``unwrapped_ball`` (``deap/benchmarks/gp.py:60-72``).  The golden
    ``c4_bench_sample`` pins 48 of these trees at the full size."""
    pset = pset_for("symreg10" if trig else "symreg10_notrig")
    trees = population(pset, "half", pop, seed, min_, max_)
    X, y = datasets.symreg10_cases(cases, seed)
    return pset, trees, X, y
