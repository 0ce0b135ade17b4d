"""The exact-integer pass on the host (CPU, no GPU): the flattener's decision
(flatten.py _int_bounds) and the interpreter's Python-number semantics
(gpeval.hip xint::run, through its host twin gpe_host_exact_eval) against
Python's own evaluation of the same trees — the reference's gp.compile path
(deap/gp.py:462-487) runs exactly that ``eval`` — and against the
reference-generated golden tests/golden/c1_int_residual.json.gz."""
import math
import operator
import random

import pytest

from conftest import load_golden
from deap_amd import _lib, build, configs, datasets, gp
from deap_amd.flatten import ExactIntRangeError, Flattener, _int_bounds
from oracle import gp_ref


def pdiv(left, right):                 # examples/gp/symbreg.py:29-33
    try:
        return left / right
    except ZeroDivisionError:
        return 1


def _pset_cmp():
    """symbreg's primitives plus lt/eq (exact int/float comparisons)."""
    ps = gp.PrimitiveSet("XI", 1)
    ps.addPrimitive(operator.add, 2)
    ps.addPrimitive(operator.sub, 2)
    ps.addPrimitive(operator.mul, 2)
    ps.addPrimitive(pdiv, 2, name="protectedDiv")
    ps.addPrimitive(operator.neg, 1)
    ps.addPrimitive(math.sin, 1)
    ps.addPrimitive(math.cos, 1)
    ps.addPrimitive(operator.lt, 2)
    ps.addPrimitive(operator.eq, 2)
    ps.renameArguments(ARG0="x")
    return ps


def _python_value(expr, ps, x):
    ctx = dict(ps.context)
    try:
        return eval("lambda x: " + expr, ctx)(x)
    except ValueError as exc:
        return exc


def _same(a, b):
    if isinstance(a, BaseException) or isinstance(b, BaseException):
        return type(a) is type(b)
    if isinstance(a, bool):
        a = int(a)
    if isinstance(a, int) or isinstance(b, int):
        return isinstance(a, int) and isinstance(b, int) and a == b
    if math.isnan(a):
        return math.isnan(b)
    return a == b and math.copysign(1.0, a) == math.copysign(1.0, b)


def _host(code, ints, x):
    try:
        return _lib.host_exact_eval(code, ints, [x])
    except ValueError as exc:
        return exc


def _check_trees(exprs, ps, xs):
    fl = Flattener(ps)
    trees = [gp.PrimitiveTree.from_string(e, ps) for e in exprs]
    idx, code, off, depth, ints, refused = fl.exact_programs(trees)
    checked = 0
    for k, j in enumerate(idx):
        prog = code[off[k]:off[k + 1]]
        for x in xs:
            exp = _python_value(str(trees[j]), ps, x)
            got = _host(prog, ints, x)
            assert _same(exp, got), (str(trees[j])[:120], x, exp, got)
            checked += 1
    return idx, refused, checked


def test_int_bound_decisions():
    ps = configs.pset_for("symbreg")
    fl = Flattener(ps)
    cases = [
        ("sub(add(18014398509481986, protectedDiv(x, sub(x, x))), "
         "18014398509481986)", True),
        ("add(18014398509481986, x)", False),      # only meets a float
        ("sub(mul(1073741824, 1073741824), 1)", False),   # folded exactly
        ("mul(add(1073741824, protectedDiv(x, sub(x, x))), "
         "add(1073741824, protectedDiv(x, sub(x, x))))", True),
        ("add(mul(x, x), protectedDiv(1, x))", False),
        ("protectedDiv(9007199254740993, add(1, protectedDiv(x, sub(x, x))))",
         True),                                    # int / int past 2**53
    ]
    for expr, need in cases:
        tree = gp.PrimitiveTree.from_string(expr, ps)
        assert _int_bounds(fl._build(tree))[0] == need, expr
        # the native flattener's candidate flag never misses one
        if need:
            assert fl.flatten([tree]).inexact == [0], expr


def test_host_exact_interpreter_matches_the_reference_golden():
    """Every tree of the reference-generated golden at every C1 point: the
    same Python number (type included) as the oracle's eval; the fitness
    from those values equals the reference's."""
    build.build()
    g = load_golden("c1_int_residual")
    ps = configs.pset_for(g["pset"])
    xs = [x / 10. for x in range(-10, 10)]
    idx, refused, checked = _check_trees(g["trees"], ps, xs)
    assert len(idx) == len(g["trees"]) - 1 and not refused
    X, T = datasets.symbreg_points()
    data = {"rows": list(zip(*X.tolist())), "terms": list(zip(*T.tolist()))}
    for s, fit in zip(g["trees"], g["fitness"]):
        kind, val = gp_ref.evaluate(s, g["pset"], data)
        assert kind == "ok"


def _rand_expr(rng, depth, big_p):
    if depth == 0 or rng.random() < 0.2:
        r = rng.random()
        if r < 0.35:
            return "x"
        if r < 0.55:
            return str(rng.randint(-3, 3))
        if r < 0.55 + big_p:
            k = rng.choice([52, 53, 54, 60, 64, 80, 100, 127, 128, 150, 200])
            return str(rng.choice([-1, 1]) * (2 ** k + rng.randint(-3, 3)))
        if r < 0.9:
            return "protectedDiv(x, sub(x, x))"          # int 1 per case
        return repr(rng.choice([0.5, -1.25, 3.0, 1e20, -0.0, 2.0 ** 60]))
    op = rng.choice(["add", "sub", "mul", "protectedDiv", "protectedDiv",
                     "neg", "lt", "eq", "sin"])
    if op in ("neg", "sin"):
        return "%s(%s)" % (op, _rand_expr(rng, depth - 1, big_p))
    return "%s(%s, %s)" % (op, _rand_expr(rng, depth - 1, big_p),
                           _rand_expr(rng, depth - 1, big_p))


def test_host_exact_interpreter_random_trees():
    """Random trees mixing ints of 2**52 .. 2**200, per-case ints, floats,
    division, comparisons, sin and neg: the interpreter returns exactly the
    Python number (int or float, the float's bits) eval gives."""
    build.build()
    ps = _pset_cmp()
    rng = random.Random(11)
    exprs = [_rand_expr(rng, rng.randint(2, 6), 0.3) for _ in range(600)]
    xs = [0.0, -0.0, 0.5, -3.0, 7.25, 1e300, float("inf"), float("nan")]
    idx, refused, checked = _check_trees(exprs, ps, xs)
    assert len(idx) > 100 and checked > 800


def test_exact_division_and_comparison_rounding():
    """int / int rounded once from the exact ratio (ties to even, 2**53 ..
    2**255 operands) and int-float comparisons decided exactly."""
    build.build()
    ps = _pset_cmp()
    one = "protectedDiv(x, sub(x, x))"
    rng = random.Random(5)
    exprs = []
    for _ in range(300):
        a = rng.randrange(1, 2 ** rng.choice([54, 60, 90, 140, 200, 250]))
        b = rng.randrange(1, 2 ** rng.choice([2, 30, 54, 100, 200]))
        exprs.append("protectedDiv(add(%d, %s), add(%d, %s))"
                     % (rng.choice([-1, 1]) * a, one, b, one))
        f = float(a)
        exprs.append("lt(add(%d, %s), %r)" % (a, one, f))
        exprs.append("eq(add(%d, %s), %r)" % (int(f) - 1, one, f))
        exprs.append("lt(%r, sub(%d, %s))" % (f, a, one))
    # halfway cases of float(int) and of the ratio
    for k in (54, 70, 120):
        for t in (1, 2, 3):
            exprs.append("add(sub(%d, %s), 0.0)" % (2 ** k + t * 2 ** (k - 53), one))
            exprs.append("protectedDiv(add(%d, %s), add(1, %s))"
                         % (2 ** k + t * 2 ** (k - 53) - 1, one, one))
    idx, refused, checked = _check_trees(exprs, ps, [0.5, -2.0])
    assert len(idx) >= 1000


def test_exact_range_is_refused():
    ps = configs.pset_for("symbreg")
    p = "add(1, 1)"
    for _ in range(9):
        p = "mul(%s, %s)" % (p, p)                     # 2**512
    tree = gp.PrimitiveTree.from_string(
        "sub(add(%s, protectedDiv(x, sub(x, x))), %s)" % (p, p), ps)
    idx, code, off, depth, ints, refused = Flattener(ps).exact_programs([tree])
    assert idx == [] and isinstance(refused[0], ExactIntRangeError)
