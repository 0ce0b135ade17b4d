"""Flattener semantics on the CPU: lower every golden tree to bytecode, run it
with the numpy mirror of the kernels (tests/bytecode_ref.py) and compare with
the reference's golden fitness."""
import math
import operator

import numpy as np
import pytest

import bytecode_ref as ref
from conftest import decode_fitness, load_golden
from deap_amd import configs, datasets, gp
from deap_amd.evaluator import pack_bitplanes
from deap_amd.flatten import ERR_CONST, ERR_SYNTAX, Flattener, Op

REL = 1e-12   # north-star fp64 tolerance (relative SSE)


def parse(trees, pset):
    return [gp.PrimitiveTree.from_string(s, pset) for s in trees]


def check_symreg(name, X, T):
    g = load_golden(name)
    pset = configs.pset_for(g["pset"])
    fl = Flattener(pset)
    batch = fl.flatten(parse(g["trees"], pset))
    for i, (tree, fit, err) in enumerate(zip(g["trees"], g["fitness"],
                                             g["error"])):
        code = batch.code[batch.offsets[i]:batch.offsets[i + 1]]
        if batch.err[i] == ERR_SYNTAX:
            got = "SyntaxError"
        elif batch.err[i] == ERR_CONST:
            got = type(batch.const_exc[i]).__name__
        else:
            Tv, verr = ref.run_f(code, X)
            try:
                got = ref.mse_from_T(Tv, verr, T)
            except OverflowError:
                got = "OverflowError"
        if err is not None:
            assert got == err, (tree, got)
            continue
        exp = decode_fitness(fit)
        assert not isinstance(got, str), (tree, got)
        if math.isnan(exp):
            assert math.isnan(got), tree
        elif math.isinf(exp) or exp == 0:
            assert got == exp, tree
        else:
            assert abs(got - exp) <= REL * abs(exp), (tree, got, exp)
    return batch


def test_flatten_c1():
    X, T = datasets.symbreg_points()
    batch = check_symreg("c1_symbreg", X, T)
    assert batch.depth.max() <= 6


def test_flatten_c1_edge_cases():
    X, T = datasets.symbreg_points()
    check_symreg("c1_edge", X, T)


def test_flatten_c4():
    g = load_golden("c4_symreg10")
    X, Y = datasets.symreg10_cases(g["data"]["n"], g["data"]["seed"])
    check_symreg("c4_symreg10", X, Y)


def test_flatten_numpy_semantics():
    """examples/gp/symbreg_numpy.py: ufunc primitives, inf/nan -> 1
    protectedDiv, sin/cos(inf) = nan, numpy.sum SSE."""
    g = load_golden("np_symbreg")
    pset = configs.pset_for("symbreg_numpy")
    X, V = datasets.symbreg_numpy_points(g["data"]["n"])
    batch = Flattener(pset).flatten(parse(g["trees"], pset))
    assert not batch.err.any()
    for i, (tree, fit) in enumerate(zip(g["trees"], g["fitness"])):
        code = batch.code[batch.offsets[i]:batch.offsets[i + 1]]
        T, _ = ref.run_f(code, X)
        got = ref.np_sse_from_T(T, V[0])
        exp = decode_fitness(fit)
        # same IEEE ops, glibc sin/cos, numpy's summation order: bit-exact
        assert got == exp or (math.isnan(exp) and math.isnan(got)), \
            (tree, got, exp)


@pytest.mark.parametrize("name,table", [("c2_mux11", datasets.mux11_table),
                                        ("c3_parity6",
                                         datasets.parity6_table)])
def test_flatten_boolean(name, table):
    g = load_golden(name)
    pset = configs.pset_for(g["pset"])
    ins, outs = table()
    planes = pack_bitplanes(ins)
    out_plane = pack_bitplanes(outs)[0]
    n = ins.shape[1]
    batch = Flattener(pset).flatten(parse(g["trees"], pset))
    for i, (tree, fit) in enumerate(zip(g["trees"], g["fitness"])):
        code = batch.code[batch.offsets[i]:batch.offsets[i + 1]]
        T = ref.run_b(code, planes)
        agree = ~(T ^ out_plane)
        hits = sum(bin(int(w)).count("1") for w in agree[: n // 32])
        if n % 32:
            hits += bin(int(agree[n // 32]) & ((1 << (n % 32)) - 1)).count("1")
        assert hits == fit, tree


def test_flatten_stgp():
    g = load_golden("c5_spambase")
    pset = configs.pset_for("spambase")
    X, L = datasets.spambase_like(g["data"]["n"], g["data"]["seed"])
    batch = Flattener(pset).flatten(parse(g["trees"], pset))
    for i, (tree, fit) in enumerate(zip(g["trees"], g["fitness"])):
        code = batch.code[batch.offsets[i]:batch.offsets[i + 1]]
        T, _ = ref.run_f(code, X)
        hits = int(((T != 0) == (L != 0)).sum())
        assert hits == fit, tree


def test_sethi_ullman_keeps_stack_shallow():
    pset = configs.pset_for("symreg10")
    trees = configs.population(pset, "half", 2000, 5, 4, 8)
    batch = Flattener(pset).flatten(trees)
    assert batch.depth.max() <= 6
    # terminals are fused into their parents: fewer words than nodes
    assert len(batch.code) < batch.length.sum() * 1.05


def test_unsupported_primitive_is_loud():
    pset = gp.PrimitiveSet("MAIN", 1)
    pset.addPrimitive(max, 2)
    with pytest.raises(NotImplementedError):
        Flattener(pset)


def test_encoding_is_what_the_kernel_reads():
    pset = configs.pset_for("symbreg")
    tree = gp.PrimitiveTree.from_string("add(mul(x, x), 1)", pset)
    b = Flattener(pset).flatten([tree])
    words = b.code.tolist()
    assert words[0] == Op.LDV                         # T = x
    assert words[1] == (Op.MUL + 1)                  # T = x * T
    assert words[2] & 0xff == Op.ADD + 2             # T = 1.0 + T
    assert (words[3], words[4]) == (0, 0x3FF00000)   # f64 1.0
    assert words[5] == Op.END


def adf_individuals(strs_list):
    psets = configs.pset_for("adf_symbreg")
    return [[gp.PrimitiveTree.from_string(s, p) for s, p in zip(strs, psets)]
            for strs in strs_list]


def test_flatten_adf_inlining():
    """examples/gp/adf_symbreg.py: ADF calls inlined (arguments evaluated
    once, unread raising arguments still evaluated); the bytecode mirror +
    Python's left-to-right sum reproduce the reference bit for bit."""
    from deap_amd.flatten import ADFFlattener
    g = load_golden("adf_symbreg")
    psets = configs.pset_for("adf_symbreg")
    X, T = datasets.adf_symbreg_points()
    batch = ADFFlattener(psets).flatten(adf_individuals(g["individuals"]))
    for i, (ind, fit, err) in enumerate(zip(g["individuals"], g["fitness"],
                                            g["error"])):
        code = batch.code[batch.offsets[i]:batch.offsets[i + 1]]
        assert batch.err[i] == 0, ind
        Tv, verr = ref.run_f(code, X)
        got = ref.mse_from_T(Tv, verr, T)
        if isinstance(got, str):
            assert got == err, (ind, got)
            continue
        assert err is None, (ind, err)
        d = Tv - T[0]
        assert sum((d * d).tolist()) == decode_fitness(fit), ind


def test_threshold_protected_division_is_not_taken_for_protectedDiv():
    """a division protected by a threshold (gplearn-style
    ``l / r if abs(r) > 1e-3 else 1``) returns 1 where the kernels divide;
    it must be refused, not lowered as protectedDiv or numpy's variant."""
    def thresh_div(left, right):
        return left / right if abs(right) > 1e-3 else 1.0
    pset = gp.PrimitiveSet("MAIN", 1)
    pset.addPrimitive(thresh_div, 2)
    pset.addPrimitive(operator.add, 2)
    with pytest.raises(NotImplementedError):
        Flattener(pset)


def test_big_int_constant_raises_without_the_exact_pass():
    """an int constant past the float range is kept for the exact
    pass (fp64), which raises OverflowError where the reference converts
    it; a run without that pass (fp32) gets the reference's OverflowError
    for the individual, not an inf-based fitness."""
    from deap_amd import _lib
    from deap_amd.evaluator import GPUEvaluator, SymbRegMSE
    pset = configs.pset_for("symbreg")
    # protectedDiv's per-case int 1 meets the constant: an exact int sum
    tree = gp.PrimitiveTree.from_string(
        "add(protectedDiv(x, sub(x, x)), %d)" % 2 ** 1050, pset)
    for precision, kept in (("fp64", True), ("fp32", False)):
        batch = Flattener(pset).flatten([tree])
        assert batch.err[0] == 0 and 0 in batch.big_const
        fake = type("E", (), {"precision": precision,
                              "spec": type("S", (), {"mode": _lib.GPE_MODE_MSE})})()
        if precision == "fp32":
            assert GPUEvaluator._load_exact(fake, batch, [tree]) == 0
            assert batch.err[0] == ERR_CONST
            assert isinstance(batch.const_exc[0], OverflowError)
    with pytest.raises(OverflowError):          # symbreg.py:60's float formula
        float(gp.compile(tree, pset)(0.5))


# lowering::Val (csrc/lower_core.h): char t, double f, int64 i, bool err_value
_VAL = np.dtype({"names": ["t", "f", "i", "err"], "formats": ["S1", "<f8", "<i8", "u1"],
                 "offsets": [0, 8, 16, 24], "itemsize": 32})


def test_read_lower_pipeline_hands_every_chunk_to_lower_add():
    """Flattener.read_lower (the chunked device lowering's native pipeline):
    every chunk's read_codes buffers reach the lower_add function in order
    (here a ctypes stand-in recording them), and the population's node
    offsets come back whole."""
    import ctypes
    from deap_amd.evaluator import GPUEvaluator
    pset = configs.pset_for("symbreg")
    pop = configs.population(pset, "half", 3000, 7, 1, 4)
    fl = Flattener(pset)
    ends = GPUEvaluator._chunk_bounds(len(pop), 1024, tail=128)
    assert ends[-1] == len(pop) and len(ends) > 3
    seen = []
    proto = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.POINTER(ctypes.c_int64), ctypes.c_int64,
                             ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64))

    def add(ctx, codes, node_off, n, evals, eph_off):
        seen.append((ctx, n, ctypes.string_at(codes, node_off[n]),
                     [node_off[i] for i in range(n + 1)],
                     [eph_off[i] for i in range(n + 1)],
                     ctypes.string_at(evals, eph_off[n] * _VAL.itemsize)))
        return 0
    cb = proto(add)
    off = np.empty(len(pop) + 1, dtype=np.int64)
    rc = fl.read_lower(pop, ends, ctypes.cast(cb, ctypes.c_void_p).value, 1234, off)
    assert rc == 0
    a = 0
    n_eph = 0
    for (ctx, n, codes, no, eo, ev), b in zip(seen, ends):
        exp = fl.read_codes(pop, a, b)
        assert ctx == 1234 and n == b - a
        assert codes == exp[0] and no == np.frombuffer(exp[1], np.int64).tolist()
        # the ephemeral values (their fields: the padding is not data)
        assert eo == np.frombuffer(exp[3], np.int64).tolist()
        got, want = np.frombuffer(ev, _VAL), np.frombuffer(exp[2], _VAL)
        for f in ("t", "f", "i", "err"):
            assert np.array_equal(got[f], want[f])
        n_eph += len(got)
        a = b
    assert n_eph > 0
    assert len(seen) == len(ends)
    lens = [len(t) for t in pop]
    assert off.tolist() == np.concatenate([[0], np.cumsum(lens)]).tolist()
    # a range [start, ends[-1]): offsets from 0; bad ends or a short offsets
    # buffer are refused before anything is read
    seen.clear()
    off2 = np.empty(2000 - 700 + 1, dtype=np.int64)
    rc = fl.read_lower(pop, [1500, 2000], ctypes.cast(cb, ctypes.c_void_p).value, 7,
                       off2, 700)
    assert rc == 0 and [x[1] for x in seen] == [800, 500]
    assert off2.tolist() == np.concatenate([[0], np.cumsum(lens[700:2000])]).tolist()
    for ends_bad, buf in (([600, 2000], off2), ([2000, 1500], off2),
                          ([1500, 3001], np.empty(3000, dtype=np.int64)),
                          ([1500, 2001], np.empty(1301, dtype=np.int64))):
        with pytest.raises(ValueError):
            fl.read_lower(pop, ends_bad, ctypes.cast(cb, ctypes.c_void_p).value, 7, buf, 700)


def test_tuples1_hit_counts_in_parallel():
    """_flatnative.tuples1 at pop 1M-scale for hit counts: the list filled
    on host threads with one shared tuple per count (reference counts raised
    once per count) equals [(int(v),) ...]; floats and non-counts take the
    per-item path."""
    import gc
    import sys
    from deap_amd import _flatnative
    v = np.random.default_rng(3).integers(0, 4602, 200000).astype(np.float64)
    out = _flatnative.tuples1(v, True)
    assert out == [(int(x),) for x in v]
    k = int(v[0])
    before = sys.getrefcount(out[0])
    assert before >= int((v == k).sum())
    del out
    gc.collect()
    f = np.linspace(0, 1, 70000)
    assert _flatnative.tuples1(f, False) == [(x,) for x in f.tolist()]
    w = v.copy()
    w[-1] = -1.0                                  # not a count: per item
    out = _flatnative.tuples1(w, True)
    assert out[-1] == (-1,) and out[:-1] == [(int(x),) for x in v[:-1]]
