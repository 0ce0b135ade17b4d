"""The exact-integer pass on the host (CPU, no GPU): the flattener's decision
(flatten.py _int_bounds) and the interpreter's Python-number semantics
(gpeval.hip xint::run, through its host twin gpe_host_exact_eval) against
Python's own evaluation of the same trees — the reference's gp.compile path
(deap/gp.py:462-487) runs exactly that ``eval`` — and against the
reference-generated golden tests/golden/c1_int_residual.json.gz."""
import math
import operator
import random

import numpy as np
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
    except (ValueError, OverflowError) as exc:
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


def _host(code, ints, x, fn=None):
    try:
        return (fn or _lib.host_exact_eval)(code, ints, [x])
    except (ValueError, OverflowError, ExactIntRangeError) as exc:
        return exc


def _check_trees(exprs, ps, xs, ranged=None):
    """Host twin of the device interpreter against Python on every tree the
    flattener sends to the exact pass.  Cases where the twin reports
    ExactIntRangeError (an int past the device's 1088 bits, which Python
    still holds) are counted in *ranged* (a list) instead.  The host
    evaluator with unbounded ints (the one the library runs for those
    programs) must give Python's number or exception at every case."""
    fl = Flattener(ps)
    trees = [gp.PrimitiveTree.from_string(e, ps) for e in exprs]
    idx, code, off, depth, ints, refused = fl.exact_programs(trees)
    checked = 0
    for k, j in enumerate(idx):
        prog = code[off[k]:off[k + 1]]
        for x in xs:
            exp = _python_value(str(trees[j]), ps, x)
            big = _host(prog, ints, x, _lib.host_bigint_eval)
            assert _same(exp, big), (str(trees[j])[:120], x, exp, big)
            got = _host(prog, ints, x)
            if isinstance(got, ExactIntRangeError) and ranged is not None:
                ranged.append((str(trees[j]), x))
                continue
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


ONE = "protectedDiv(x, sub(x, x))"          # int 1 at every finite x


def _big(k):
    """add(2**k, 1 per case): a per-case int near 2**k (not foldable)."""
    return "add(%d, %s)" % (2 ** k, ONE)


def test_ints_past_2_255_are_evaluated_exactly():
    """Round 3 refused any individual whose ints could reach 2**255; the
    pass now holds 1088 bits and evaluates them as Python does."""
    build.build()
    ps = configs.pset_for("symbreg")
    p = "add(1, 1)"
    for _ in range(9):
        p = "mul(%s, %s)" % (p, p)                     # 2**512
    exprs = ["sub(add(%s, %s), %s)" % (p, ONE, p),      # exactly 1
             "mul(%s, %s)" % (_big(300), _big(500)),
             "sub(mul(%s, %s), mul(%s, %s))" % (_big(500), _big(500),
                                                _big(500), _big(500))]
    idx, refused, checked = _check_trees(exprs, ps, [0.5, -3.0, 0.0])
    assert idx == [0, 1, 2] and not refused and checked == 9
    code_ok = _lib.host_exact_eval
    fl = Flattener(ps)
    t = gp.PrimitiveTree.from_string(exprs[0], ps)
    i, code, off, depth, ints, _ = fl.exact_programs([t])
    assert code_ok(code[off[0]:off[1]], ints, [0.5]) == 1


def test_float_of_a_huge_int_raises_overflow_like_the_reference():
    """float(int) at or past 2**1024 (a mixed int-float operation, sin of an
    int, protectedDiv converting its operands) and int / int past the float
    range raise OverflowError, as CPython does; exact int arithmetic and
    int-float comparisons of such ints do not."""
    build.build()
    ps = _pset_cmp()
    sq = "mul(%s, %s)" % (_big(520), _big(520))        # ~2**1040, per case
    exprs = ["add(%s, x)" % sq,                        # OverflowError
             "mul(x, %s)" % sq,
             "sin(%s)" % sq,
             "protectedDiv(%s, add(1, %s))" % (sq, ONE),   # int / int: too large
             "protectedDiv(x, %s)" % sq,               # float / int: converts
             "protectedDiv(%s, sub(x, x))" % sq,       # converts before the 0 test
             "protectedDiv(add(7, %s), %s)" % (ONE, sq),   # tiny ratio: 0.0
             "protectedDiv(add(%d, %s), mul(%s, %s))" % (2 ** 10, ONE, _big(540),
                                                         _big(540)),  # subnormal
             "lt(%s, 1e308)" % sq, "eq(%s, %s)" % (sq, sq),
             "sub(%s, %s)" % (sq, sq),
             "add(sub(%s, %s), x)" % (sq, sq),
             "add(%d, %s)" % (2 ** 1023, ONE),         # fine: < 2**1024
             "add(add(%d, %s), 0.5)" % (2 ** 1023, ONE),
             "add(sub(mul(%d, 2), %s), 0.5)" % (2 ** 1023, ONE)]   # 2**1024 - 1
    xs = [0.5, -3.0, 0.0]
    idx, refused, checked = _check_trees(exprs, ps, xs)
    assert len(idx) == len(exprs) and not refused
    assert checked == len(exprs) * len(xs)
    over = sum(isinstance(_python_value(e, ps, 0.5), OverflowError)
               for e in exprs)
    assert over >= 7


def test_ints_past_1088_bits_are_evaluated_on_the_host():
    """Ints past the device's 1088 bits (its twin reports the range) get
    the reference's value from the host evaluator: products that cancel,
    exact true division of huge ints, and constants past 2**1088."""
    build.build()
    ps = _pset_cmp()
    huge = "mul(mul(%s, %s), %s)" % (_big(400), _big(400), _big(400))  # ~2**1200
    exprs = ["sub(%s, %s)" % (huge, huge),                    # 0
             "protectedDiv(%s, %s)" % (huge, huge),           # 1.0
             "protectedDiv(%s, add(%s, 1))" % (huge, huge),   # 1.0 (rounded)
             "protectedDiv(%s, %s)" % (huge, _big(100)),      # OverflowError
             "sub(add(%d, %s), %d)" % (2 ** 1100, ONE, 2 ** 1100),  # 1
             "lt(add(%d, %s), x)" % (-2 ** 1500, ONE),        # True
             "add(mul(%s, %s), x)" % (huge, huge)]            # OverflowError
    ranged = []
    idx, refused, checked = _check_trees(exprs, ps, [0.5, 2.0], ranged)
    assert idx == list(range(len(exprs))) and not refused
    assert len(ranged) == 2 * len(exprs) and checked == 0
    assert _python_value(exprs[0], ps, 0.5) == 0      # the reference's value
    assert _python_value(exprs[1], ps, 0.5) == 1.0
    assert isinstance(_python_value(exprs[3], ps, 0.5), OverflowError)
    assert _python_value(exprs[4], ps, 0.5) == 1


def test_int_table_has_no_size_limit():
    """Round 4 refused the individuals past 65,535 distinct int constants
    in one exact batch; the table's row index now sits in the constant's two
    data words: a program reading row 70,000 of a 70,001-row table."""
    build.build()
    from deap_amd.flatten import IntTable
    ps = configs.pset_for("symbreg")
    fl = Flattener(ps)
    t = gp.PrimitiveTree.from_string("sub(add(%d, %s), 5)" % (2 ** 60, ONE), ps)
    idx, code, off, depth, ints, refused = fl.exact_programs([t])
    assert idx == [0] and not refused and ints.values == [2 ** 60, 5]
    vals = list(range(70001))
    vals[70000] = 2 ** 60 + 7                         # the first constant's row
    vals[1], vals[5] = 5, 1                           # the second's (5)
    table = IntTable({v: r for r, v in enumerate(vals)})
    prog = np.array(code[off[0]:off[1]], dtype=np.uint32)
    # the first int constant (2**60): point it at row 70000
    k0 = next(k for k in range(len(prog)) if prog[k] >> 16 == 1)
    assert prog[k0 + 1] == 0 and prog[k0 + 2] == 0
    prog[k0 + 1] = 70000
    for fn in (_lib.host_exact_eval, _lib.host_bigint_eval):
        assert fn(prog, table, [0.5]) == 2 ** 60 + 7 + 1 - 5


def test_random_trees_with_huge_ints():
    """Random trees with ints up to 2**1000 and products past 2**1024:
    values, OverflowErrors and ValueErrors exactly as Python's, from the
    device interpreter's twin (cases past its 1088 bits reported) and from
    the host evaluator (every case)."""
    build.build()
    ps = _pset_cmp()
    rng = random.Random(23)

    def expr(depth):
        if depth == 0 or rng.random() < 0.2:
            r = rng.random()
            if r < 0.3:
                return "x"
            if r < 0.6:
                k = rng.choice([60, 200, 400, 520, 700, 1000])
                return "add(%d, %s)" % (rng.choice([-1, 1]) * 2 ** k, ONE)
            if r < 0.8:
                return ONE
            return repr(rng.choice([0.5, -1.25, 1e300, 2.0 ** 1000]))
        op = rng.choice(["add", "sub", "mul", "mul", "protectedDiv", "neg",
                         "lt", "eq", "sin"])
        if op in ("neg", "sin"):
            return "%s(%s)" % (op, expr(depth - 1))
        return "%s(%s, %s)" % (op, expr(depth - 1), expr(depth - 1))
    exprs = [expr(rng.randint(2, 5)) for _ in range(400)]
    ranged = []
    idx, refused, checked = _check_trees(exprs, ps, [0.5, -3.0, 0.0, 1e300],
                                         ranged)
    assert len(idx) > 150 and checked > 500
    assert 0 < len(ranged) < checked / 10


def test_host_bigint_evaluator_matches_the_int_huge_golden():
    """tests/golden/c1_int_huge (reference-generated: ints past 2**1088 that
    cancel, divide exactly, or overflow only in the error formula; a folded
    constant of 2**1200): the host evaluator's values at every C1 point give
    the reference's fitness (symbreg.py:60-61's fsum formula) or its
    exception."""
    build.build()
    g = load_golden("c1_int_huge")
    ps = configs.pset_for(g["pset"])
    fl = Flattener(ps)
    trees = [gp.PrimitiveTree.from_string(s, ps) for s in g["trees"]]
    idx, code, off, depth, ints, refused = fl.exact_programs(trees)
    assert idx == list(range(len(trees))) and not refused
    xs = [x / 10. for x in range(-10, 10)]
    for k, (fit, err) in enumerate(zip(g["fitness"], g["error"])):
        prog = code[off[k]:off[k + 1]]
        try:
            vals = [_lib.host_bigint_eval(prog, ints, [x]) for x in xs]
            got = math.fsum((v - x ** 4 - x ** 3 - x ** 2 - x) ** 2
                            for v, x in zip(vals, xs)) / len(xs)
        except OverflowError:
            assert err == "OverflowError", g["trees"][k][:80]
            continue
        assert err is None and got == float.fromhex(fit), (g["trees"][k][:80], got)
