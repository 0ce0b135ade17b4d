"""Pin the oracle (oracle/gp_ref.py) to the reference's own outputs.

Every committed golden vector was produced by running the reference
(tests/golden/make_golden.py); the CPU restatement must reproduce all of them
bit for bit.
"""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, decode_fitness, load_golden
from deap_amd import datasets
from oracle import gp_ref


def data_for(spec):
    kind = spec["data"]["kind"]
    d = spec["data"]
    if kind == "symbreg_points":
        X, T = datasets.symbreg_points()
        return {"rows": list(zip(*X.tolist())), "terms": list(zip(*T.tolist()))}
    if kind == "symreg10_cases":
        X, Y = datasets.symreg10_cases(d["n"], d["seed"])
        return {"rows": list(zip(*X.tolist())), "terms": list(zip(*Y.tolist()))}
    if kind == "mux11_table":
        ins, outs = datasets.mux11_table()
        return {"inputs": [list(map(int, c)) for c in ins.T],
                "outputs": list(map(int, outs))}
    if kind == "parity6_table":
        ins, outs = datasets.parity6_table()
        return {"inputs": [list(map(int, c)) for c in ins.T],
                "outputs": list(map(int, outs))}
    if kind == "spambase_like":
        X, L = datasets.spambase_like(d["n"], d["seed"])
        return {"rows": list(zip(*X.tolist())), "labels": list(map(int, L))}
    if kind == "spambase_csv":
        X, L = datasets.spambase_csv(os.path.join(GOLDEN, d["file"]))
        return {"rows": list(zip(*X.tolist())), "labels": list(map(int, L))}
    if kind == "symbreg_numpy_points":
        X, V = datasets.symbreg_numpy_points(d["n"])
        return {"samples": X[0], "values": V[0]}
    if kind == "adf_symbreg_points":
        X, T = datasets.adf_symbreg_points()
        return {"points": X[0].tolist(), "targets": T[0].tolist()}
    raise KeyError(kind)


@pytest.mark.parametrize("name", ["c1_symbreg", "c1_edge", "c1_int_residual",
                                  "c2_mux11",
                                  "c3_parity6", "c4_symreg10",
                                  "c5_spambase", "c5_spambase_real",
                                  "np_symbreg"])
def test_oracle_matches_reference_goldens(name):
    g = load_golden(name)
    data = data_for(g)
    for tree, fit, err in zip(g["trees"], g["fitness"], g["error"]):
        kind, val = gp_ref.evaluate(tree, g["pset"], data)
        if err is not None:
            assert (kind, val) == ("err", err), tree
        else:
            assert kind == "ok", (tree, val)
            exp = decode_fitness(fit)
            if isinstance(exp, float) and math.isnan(exp):
                assert math.isnan(val)
            else:
                assert val == exp, tree


def test_oracle_matches_reference_deep_core_golden_sample():
    """Every 8th tree of the deep-core golden (6..12 stack slots, 4,096
    cases; the full set is checked on the GPU) through the oracle."""
    g = load_golden("c4_deep_core")
    data = data_for(g)
    for tree, fit, err in list(zip(g["trees"], g["fitness"], g["error"]))[::8]:
        kind, val = gp_ref.evaluate(tree, g["pset"], data)
        if err is not None:
            assert (kind, val) == ("err", err), tree[:80]
        else:
            exp = decode_fitness(fit)
            assert kind == "ok" and (val == exp or (math.isnan(val) and
                                                    math.isnan(exp))), tree[:80]


def test_oracle_matches_reference_adf_goldens():
    g = load_golden("adf_symbreg")
    data = data_for(g)
    for ind, fit, err in zip(g["individuals"], g["fitness"], g["error"]):
        kind, val = gp_ref.evaluate(ind, "adf_symbreg", data)
        if err is not None:
            assert (kind, val) == ("err", err), ind
        else:
            assert (kind, val) == ("ok", decode_fitness(fit)), ind


def test_oracle_1m_subset():
    g = load_golden("c4_symreg10_1m")
    X, Y = datasets.symreg10_cases(g["data"]["n"], g["data"]["seed"])
    import hashlib
    assert hashlib.sha256(X.tobytes()).hexdigest() == g["data"]["sha256_X"]
    assert hashlib.sha256(Y.tobytes()).hexdigest() == g["data"]["sha256_y"]
    data = {"rows": list(zip(*X.tolist())), "terms": list(zip(*Y.tolist()))}
    for tree, fit in list(zip(g["trees"], g["fitness"]))[:2]:
        kind, val = gp_ref.evaluate(tree, "symreg10", data)
        assert kind == "ok" and val == decode_fitness(fit)


def test_golden_data_checksums():
    import hashlib
    for name in ("c4_symreg10", "c5_spambase", "np_symbreg"):
        g = load_golden(name)
        d = g["data"]
        if d["kind"] == "symbreg_numpy_points":
            X, V = datasets.symbreg_numpy_points(d["n"])
            assert hashlib.sha256(V.tobytes()).hexdigest() == \
                d["sha256_values"]
        elif d["kind"] == "symreg10_cases":
            X, Y = datasets.symreg10_cases(d["n"], d["seed"])
            assert hashlib.sha256(Y.tobytes()).hexdigest() == d["sha256_y"]
        else:
            X, L = datasets.spambase_like(d["n"], d["seed"])
            assert hashlib.sha256(L.tobytes()).hexdigest() == d["sha256_labels"]
        assert hashlib.sha256(X.tobytes()).hexdigest() == d["sha256_X"]


def test_truth_tables_match_reference_construction():
    # multiplexer.py:37-54 / parity.py:31-47 restated literally
    ins, outs = datasets.mux11_table()
    for i in (0, 1, 5, 777, 2047):
        value, divisor = i, 2 ** 11
        bits = []
        for _ in range(11):
            divisor /= 2
            if value >= divisor:
                bits.append(1); value -= divisor
            else:
                bits.append(0)
        assert list(ins[:, i]) == bits
        idx = 3 + sum(k * 2 ** j for j, k in enumerate(bits[:3]))
        assert outs[i] == bits[idx]
    ins, outs = datasets.parity6_table()
    assert outs.sum() == 32 and outs[0] == 1 and outs[1] == 0


def test_bench_sample_pins_the_bench_population_and_reference_target():
    """c4_bench_sample.json.gz was computed by the reference on bench.py's
    own workload: the 48 trees are those bench.py generates at their
    indices, X is bench.py's X, and datasets.unwrapped_ball_py gives the
    reference's unwrapped_ball (deap/benchmarks/gp.py:60-72) bit for bit."""
    import hashlib
    from deap_amd import configs
    g = load_golden("c4_bench_sample")
    d, p = g["data"], g["population"]
    pset, trees, X, y = configs.headline_c4(p["n"], d["n"], d["seed"],
                                            p["min"], p["max"])
    assert [str(trees[i]) for i in g["index"]] == g["trees"]
    assert hashlib.sha256(X.tobytes()).hexdigest() == d["sha256_X"]
    assert hashlib.sha256(y[0].tobytes()).hexdigest() == d["sha256_y_ref"]
    assert sum(g["redo"]) >= 16 and all(e is None for e in g["error"])


def test_oracle_matches_bench_sample_golden_at_full_size():
    """The oracle restatement reproduces the reference's full-size fitness
    for two of the golden's trees (one on the redo path) bit for bit."""
    from deap_amd import configs
    g = load_golden("c4_bench_sample")
    d = g["data"]
    X, y = datasets.symreg10_cases(d["n"], d["seed"])
    data = {"rows": list(zip(*X.tolist())), "terms": [(v,) for v in y[0]]}
    for k in (0, g["redo"].index(True)):
        kind, exp = gp_ref.evaluate(g["trees"][k], "symreg10", data)
        assert kind == "ok"
        assert exp == decode_fitness(g["fitness"][k])


def _full_fixture(name):
    import base64
    g = load_golden(name)
    fit = np.frombuffer(base64.b64decode(g["fitness_f64_b64"]), dtype="<f8")
    assert len(fit) == g["n_trees"]
    return g, fit


def test_full_fixtures_pin_their_populations_and_data():
    """c4_bench_full_2e16 (all 65,536 headline trees at the first 2^16 bench
    cases) and c4_evolved_ref (all 4,096 evolved trees at 4,096 cases) were
    computed by the reference (tests/golden/_bench_full.py) on exactly the
    trees and cases the GPU tests regenerate: tree-string and data hashes."""
    import gzip
    import hashlib
    import json
    from deap_amd import configs
    g, fit = _full_fixture("c4_bench_full_2e16")
    p, c = g["population"], g["cases"]
    _, trees, _, _ = configs.headline_c4(p["n"], 128, p["seed"], p["min"], p["max"])
    assert hashlib.sha256("\n".join(str(t) for t in trees).encode()).hexdigest() \
        == g["sha256_trees"]
    X, y = datasets.symreg10_cases(c["first"], c["seed"])
    assert hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest() == \
        g["data"]["sha256_X"]
    assert hashlib.sha256(y[0].tobytes()).hexdigest() == g["data"]["sha256_y_ref"]
    assert np.isfinite(fit).sum() + len(g["error"]) >= len(fit) - 1
    g2, _ = _full_fixture("c4_evolved_ref")
    with gzip.open(os.path.join(GOLDEN, "c4_evolved.json.gz"), "rt") as fh:
        strs = json.load(fh)["trees"]
    assert hashlib.sha256("\n".join(strs).encode()).hexdigest() == g2["sha256_trees"]


def test_oracle_matches_full_fixtures_on_a_sample():
    """The oracle restatement reproduces the reference's fitness, bit for
    bit, for a sample of the full fixtures' trees (6 headline trees at 2^16
    cases, 24 evolved trees at 4,096 cases)."""
    import gzip
    import json
    from deap_amd import configs
    g, fit = _full_fixture("c4_bench_full_2e16")
    p, c = g["population"], g["cases"]
    _, trees, _, _ = configs.headline_c4(p["n"], 128, p["seed"], p["min"], p["max"])
    X, y = datasets.symreg10_cases(c["first"], c["seed"])
    rows, terms = list(zip(*X.tolist())), [(v,) for v in y[0].tolist()]
    for i in np.random.default_rng(2).choice(len(trees), 6, replace=False).tolist():
        assert gp_ref.eval_symreg_mse(str(trees[i]), "symreg10", rows, terms) == fit[i]
    g, fit = _full_fixture("c4_evolved_ref")
    with gzip.open(os.path.join(GOLDEN, "c4_evolved.json.gz"), "rt") as fh:
        strs = json.load(fh)["trees"]
    X, y = datasets.symreg10_cases(4096, 2024)
    rows, terms = list(zip(*X.tolist())), [(v,) for v in y[0].tolist()]
    for i in np.random.default_rng(3).choice(len(strs), 24, replace=False).tolist():
        assert gp_ref.eval_symreg_mse(strs[i], "symreg10", rows, terms) == fit[i]


def test_full_fixture_notes_are_pow_misrounds():
    """Every tree c4_full_notes.json lets differ from the reference (the
    device's exact-square sum, scripts/r06_classify_full.py) really is one
    where the reference's d ** 2 (glibc pow) misrounds: the oracle's
    math.fsum(d ** 2) / n is the fixture's value and math.fsum(d * d) / n
    the noted one, and the two differ."""
    import gzip
    import json
    from deap_amd import configs
    with open(os.path.join(GOLDEN, "c4_full_notes.json")) as fh:
        notes = json.load(fh)
    g, fit = _full_fixture("c4_bench_full_2e16")
    p, c = g["population"], g["cases"]
    _, trees, _, _ = configs.headline_c4(p["n"], 128, p["seed"], p["min"], p["max"])
    X, y = datasets.symreg10_cases(c["first"], c["seed"])
    with gzip.open(os.path.join(GOLDEN, "c4_evolved.json.gz"), "rt") as fh:
        evolved = json.load(fh)["trees"]
    Xe, ye = datasets.symreg10_cases(4096, 2024)
    g2, fit2 = _full_fixture("c4_evolved_ref")
    for name, strs, Xs, ys, fx in (("c4_bench_full_2e16", [str(t) for t in trees], X, y, fit),
                                   ("c4_evolved_ref", evolved, Xe, ye, fit2)):
        rows = list(zip(*Xs.tolist()))
        for i, n in sorted(notes[name].items()):
            i = int(i)
            assert n["why"] == "pow"
            f = gp_ref.compile_expr(strs[i], "symreg10")
            d = [f(*r) - t for r, t in zip(rows, ys[0].tolist())]
            ref = math.fsum(v ** 2 for v in d) / len(d)
            mul = math.fsum(v * v for v in d) / len(d)
            assert ref == fx[i] and mul == float.fromhex(n["mul"]) and ref != mul
