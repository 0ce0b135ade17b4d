"""The native flattener (csrc/flatten_native.cpp) emits exactly the words of
the Python specification (Flattener.flatten_py) — on every golden set, on
fresh populations of every primitive set, with trig-leaf columns, on pickled
trees (nodes found by name, not identity) and on trees it declines."""
import os
import pickle
import time

import numpy as np
import pytest

from conftest import load_golden
from deap_amd import configs, gp
from deap_amd.flatten import Flattener

GOLDEN = ["c1_symbreg", "c1_edge", "c2_mux11", "c3_parity6", "c4_symreg10",
          "c5_spambase", "np_symbreg"]


def same(a, b):
    assert len(a) == len(b)
    assert np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.code, b.code)
    assert np.array_equal(a.depth, b.depth)
    assert np.array_equal(a.length, b.length)
    assert np.array_equal(a.err, b.err)
    assert sorted(a.const_exc) == sorted(b.const_exc)
    for i in a.const_exc:
        assert type(a.const_exc[i]) is type(b.const_exc[i])
    assert list(a.inexact) == list(b.inexact)


@pytest.mark.parametrize("name", GOLDEN)
def test_native_matches_python_on_goldens(name):
    g = load_golden(name)
    pset = configs.pset_for(g["pset"])
    trees = [gp.PrimitiveTree.from_string(s, pset) for s in g["trees"]]
    fl = Flattener(pset)
    same(fl.flatten(trees), fl.flatten_py(trees))


@pytest.mark.parametrize("pname,gen,lo,hi", [
    ("symbreg", "half", 1, 6), ("symreg10", "half", 4, 8),
    ("mux11", "full", 2, 4), ("parity6", "full", 3, 5),
    ("spambase", "half", 2, 6), ("symbreg_numpy", "half", 1, 6)])
def test_native_matches_python_on_populations(pname, gen, lo, hi):
    pset = configs.pset_for(pname)
    pop = configs.population(pset, gen, 3000, 11, lo, hi)
    fl = Flattener(pset)
    same(fl.flatten(pop), fl.flatten_py(pop))


def test_native_trig_leaves_and_pickled_trees():
    pset = configs.pset_for("symreg10")
    pop = configs.population(pset, "half", 2000, 5, 2, 7)
    fl = Flattener(pset, trig_leaves=[0, 2, 3, 7, 9])
    same(fl.flatten(pop), fl.flatten_py(pop))
    thawed = pickle.loads(pickle.dumps(pop))       # new node objects
    assert thawed[0][0] is not pop[0][0]
    same(fl.flatten(thawed), fl.flatten_py(pop))


def test_declined_trees_are_spliced_from_the_python_path():
    pset = configs.pset_for("symbreg")
    # integers beyond int64 and beyond 2**53 in folded constant subtrees
    texts = ["add(x, mul(mul(mul(-1, -1), 4611686018427387904), 4))",
             "mul(x, mul(4294967296, 4294967296))",
             "add(x, 1)", "cos(mul(x, x))"]
    trees = [gp.PrimitiveTree.from_string(t, pset) for t in texts]
    fl = Flattener(pset)
    same(fl.flatten(trees), fl.flatten_py(trees))


def test_native_is_much_faster_than_python():
    pset = configs.pset_for("symreg10")
    pop = configs.population(pset, "half", 4000, 3, 4, 8)
    fl = Flattener(pset)
    fl.flatten(pop[:10])
    t0 = time.perf_counter()
    fl.flatten(pop)
    t_nat = time.perf_counter() - t0
    t0 = time.perf_counter()
    fl.flatten_py(pop)
    t_py = time.perf_counter() - t0
    assert t_nat * 5 < t_py, (t_nat, t_py)


def test_threaded_lowering_matches_python_with_gil_fallback_mixed_in():
    """>= 4096 trees per worker engages the threads; pickled trees (nodes
    found by name, read by the calling thread) are interleaved with them."""
    pset = configs.pset_for("symreg10")
    pop = configs.population(pset, "half", 20000, 9, 2, 6)
    thawed = pickle.loads(pickle.dumps(pop[::97]))
    mixed = list(pop)
    for j, t in zip(range(0, len(mixed), 97), thawed):
        mixed[j] = t
    fl = Flattener(pset)
    same(fl.flatten(mixed), fl.flatten_py(pop))
    spam = configs.pset_for("spambase")
    pop5 = configs.population(spam, "half", 12000, 4, 1, 3)
    fl5 = Flattener(spam)
    same(fl5.flatten(pop5), fl5.flatten_py(pop5))


def test_thread_pool_reused_across_calls():
    """The native passes run on one persistent host-thread pool
    (csrc/host_pool.h): back-to-back calls — and calls at other thread
    counts — give the same words as the first."""
    pset = configs.pset_for("symreg10")
    pop = configs.population(pset, "half", 24000, 5, 2, 6)
    fl = Flattener(pset)
    ref = fl.flatten_py(pop)
    old = os.environ.get("OMP_NUM_THREADS")
    try:
        for t in ("8", "3", "16", "1", "8"):
            os.environ["OMP_NUM_THREADS"] = t
            same(fl.flatten(pop), ref)
    finally:
        if old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = old


LOWER_SETS = [("c1_symbreg", None), ("c1_edge", None), ("c2_mux11", None),
              ("c3_parity6", None), ("c4_symreg10", None),
              ("c5_spambase", None), ("symbreg_numpy", (2000, 2, 8)),
              ("symreg10", (4000, 1, 12)), ("parity6", (2000, 2, 10)),
              ("spambase", (3000, 2, 8))]


@pytest.mark.parametrize("name,pop", LOWER_SETS)
@pytest.mark.parametrize("leaves", [False, True])
def test_read_codes_lowering_equals_native_flatten(name, pop, leaves):
    """The device-lowering path on the host: read_codes (per-node pset codes,
    ephemeral values) lowered by lowering::lower — the function the
    lower_trees kernel runs — gives the native flattener's words, depth,
    error codes and flags, tree by tree."""
    from deap_amd import _flatnative
    if pop is None:
        g = load_golden(name)
        pset = configs.pset_for(g["pset"])
        trees = [gp.PrimitiveTree.from_string(s, pset) for s in g["trees"]]
    else:
        pset = configs.pset_for(name)
        n, lo, hi = pop
        trees = configs.population(pset, "half", n, 11, lo, hi)
    f = Flattener(pset)
    if leaves:
        if f.machine != 0 or not f.spec.has_trig:
            pytest.skip("no sin/cos leaves on this pset")
        f = Flattener(pset, trig_leaves=range(len(f.spec.arg_index)))
    r = f.read_codes(trees)
    assert r is not None
    code, off, depth, err, status = _flatnative.lower_codes(
        f._native_handle()[0], *r)
    code = np.frombuffer(code, np.uint32)
    off = np.frombuffer(off, np.int64)
    status = np.frombuffer(status, np.uint8)
    cap = f._native_handle()[0]
    declined = _flatnative.flatten(cap, trees)[6]
    # trees whose constant folding needs Python (ints past int64) are
    # declined by both, and the evaluator lowers such batches on the host
    assert np.flatnonzero(status & 1).tolist() == sorted(declined)
    host = f.flatten(trees)
    keep = np.flatnonzero((status & 1) == 0)
    hoff = host.offsets
    for i in keep.tolist():
        assert np.array_equal(code[off[i]:off[i + 1]],
                              host.code[hoff[i]:hoff[i + 1]]), i
    assert np.array_equal(np.frombuffer(depth, np.int32)[keep],
                          host.depth[keep])
    assert np.array_equal(np.frombuffer(err, np.uint8)[keep], host.err[keep])
    ok = set(keep.tolist())
    assert np.flatnonzero(status & 4).tolist() == \
        sorted(i for i in host.const_exc if i in ok)
    assert np.flatnonzero(status & 2).tolist() == \
        [i for i in host.inexact if i in ok]
    assert np.array_equal(np.diff(np.frombuffer(r[1], np.int64)), host.length)


def test_packed_records_decline_trees_past_16_bit_indices():
    """The device's packed records hold node indices in 16 bits: a tree of
    more than 65,535 nodes is declined by the device path (the evaluator
    then lowers the batch on the host), and lowered normally on the host."""
    from deap_amd import _flatnative
    pset = configs.pset_for("symreg10")
    add = pset.mapping["add"]
    args = pset.arguments

    def full(d):                       # prefix order of a full binary tree
        if d == 0:
            return [pset.mapping[args[0]]]
        return [add] + full(d - 1) + full(d - 1)
    big = gp.PrimitiveTree(full(16))   # 131,071 nodes, height 16
    small = gp.PrimitiveTree.from_string("add(ARG1, ARG2)", pset)
    f = Flattener(pset)
    r = f.read_codes([big, small])
    assert r is not None
    code, off, depth, err, status = _flatnative.lower_codes(
        f._native_handle()[0], *r)
    status = np.frombuffer(status, np.uint8)
    assert status[0] & 1 and status[1] == 0
    host = f.flatten([big, small])
    assert host.length[0] > 65535 and host.err[0] == 0
