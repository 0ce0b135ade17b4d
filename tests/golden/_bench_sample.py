#!/usr/bin/env python3
"""Golden fitness for a sample of bench.py's own headline population.

bench.py times config 4 on 65,536 trees (``configs.population(pset, "half",
65536, 2024, 4, 8)``) x 2**20 cases (X ~ U(-1, 1) from
``default_rng(2024)``).  This script picks 48 of those trees — 16 whose
sin/cos arguments leave the asm core's range (|x| >= 2^40 or inf/nan: the
tile-level redo path) and 32 others — and evaluates them with the
REFERENCE at all 2**20 cases:

* the target is the reference's ``deap/benchmarks/gp.py:60-72``
  ``unwrapped_ball`` over every row (its sha256 is stored; the GPU test and
  bench.py check that ``datasets.unwrapped_ball_py`` gives the same bits);
* fitness is the reference's ``gp.compile`` (``deap/gp.py:462-487``) and
  the ``examples/gp/symbreg.py:60-61`` loop shape
  (``math.fsum((func(*x) - y)**2 ...) / len(points)``).

Run in the build container only (needs the 2to3 copy of the reference,
``make_oracle_copy.sh``): ``python3 tests/golden/_bench_sample.py``.
Writes ``c4_bench_sample.json.gz``.
"""
import gzip
import hashlib
import json
import math
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ORACLE_COPY = os.environ.get("DEAP_ORACLE_COPY", "/tmp/deap_oracle")
sys.path.insert(0, HERE)
sys.path.insert(1, REPO)

SEED, POP, CASES, MIN_D, MAX_D = 2024, 65536, 2 ** 20, 4, 8
N_REDO, N_OTHER = 16, 32
LIM = 2.0 ** 40


def bench_data():
    """bench.py's X (variable-planar) for the full case set."""
    rng = np.random.default_rng(SEED)
    return np.ascontiguousarray(rng.uniform(-1.0, 1.0, size=(CASES, 10)).T)


def bench_population():
    from deap_amd import configs
    pset = configs.pset_for("symreg10")
    return configs.population(pset, "half", POP, SEED, MIN_D, MAX_D)


def max_trig_arg(tree, X):
    """numpy evaluation of one tree, returning max |sin/cos argument|
    (inf for inf/nan arguments) — only to find redo-path programs."""
    from deap_amd import gp as cgp
    worst = [0.0]

    def ev(i):
        node = tree[i]
        if isinstance(node, cgp.Terminal):
            v = node.value
            if isinstance(v, str):
                return X[int(v[3:])], i + 1
            return np.full(X.shape[1], float(v)), i + 1
        vals, j = [], i + 1
        for _ in range(node.arity):
            v, j = ev(j)
            vals.append(v)
        n = node.name
        with np.errstate(all="ignore"):
            if n == "add":
                return vals[0] + vals[1], j
            if n == "sub":
                return vals[0] - vals[1], j
            if n == "mul":
                return vals[0] * vals[1], j
            if n == "protectedDiv":
                z = vals[1] == 0
                return np.where(z, 1.0, vals[0] / np.where(z, 1.0, vals[1])), j
            if n == "neg":
                return -vals[0], j
            a = np.abs(vals[0])
            bad = ~np.isfinite(a)
            worst[0] = max(worst[0], float(np.inf if bad.any() else a.max()))
            return (np.sin if n == "sin" else np.cos)(vals[0]), j
        raise KeyError(n)
    ev(0)
    return worst[0]


def _scan(args):
    lo, hi, n_cases = args
    X = bench_data()[:, :n_cases]
    pop = bench_population()
    return [(i, max_trig_arg(pop[i], X)) for i in range(lo, hi)]


def _ref_eval(tree_str):
    sys.path.insert(0, ORACLE_COPY)
    from deap import gp  # the reference (2to3 copy)
    import make_golden
    pset = make_golden.arith_pset(10, False)
    rows, ys = _REF["rows"], _REF["y"]

    def mse():
        func = gp.compile(tree_str, pset)
        return math.fsum((func(*x) - y) ** 2 for x, y in zip(rows, ys)) \
            / len(rows)
    val, err = make_golden.run(mse)
    return make_golden.enc(val), err


_REF = {}


def main():
    pop = bench_population()
    strs = [str(t) for t in pop]
    # 1. redo candidates on the first 2^14 cases (8 processes)
    n_scan = 2 ** 14
    chunks = [(lo, min(POP, lo + 2048), n_scan) for lo in range(0, POP, 2048)]
    with mp.get_context("fork").Pool(8) as pool:
        scanned = [r for part in pool.map(_scan, chunks) for r in part]
    cand = [i for i, m in scanned if not (m < LIM)]
    print("redo candidates in %d cases: %d" % (n_scan, len(cand)))
    rng = np.random.default_rng(99)
    redo = sorted(rng.choice(cand, N_REDO, replace=False).tolist())
    rest = [i for i in range(POP) if i not in set(cand)]
    other = sorted(rng.choice(rest, N_OTHER, replace=False).tolist())
    idx = sorted(redo + other)
    # 2. the full case set: reference target, then reference fitness
    X = bench_data()
    sys.path.insert(0, ORACLE_COPY)
    from deap.benchmarks import gp as bgp   # reference benchmarks/gp.py
    rows = list(zip(*[col.tolist() for col in X]))
    y_ref = np.array([bgp.unwrapped_ball(r) for r in rows])
    from deap_amd import datasets
    y_ours = datasets.unwrapped_ball_py(X)
    assert y_ours.tobytes() == y_ref.tobytes(), "datasets y != reference y"
    full_max = [max_trig_arg(pop[i], X) for i in idx]
    _REF["rows"], _REF["y"] = rows, y_ref.tolist()
    with mp.get_context("fork").Pool(8) as pool:
        res = pool.map(_ref_eval, [strs[i] for i in idx], chunksize=1)
    payload = {
        "pset": "symreg10",
        "data": {"kind": "bench", "seed": SEED, "n": CASES,
                 "sha256_X": hashlib.sha256(X.tobytes()).hexdigest(),
                 "sha256_y_ref": hashlib.sha256(y_ref.tobytes()).hexdigest(),
                 "y": "reference deap/benchmarks/gp.py:60-72 unwrapped_ball"},
        "population": {"generator": "half", "n": POP, "seed": SEED,
                       "min": MIN_D, "max": MAX_D},
        "index": idx, "trees": [strs[i] for i in idx],
        "redo": [i in set(redo) for i in idx],
        "max_trig_arg": [m if m < LIM else "inf" if math.isinf(m) else m
                         for m in full_max],
        "fitness": [r[0] for r in res], "error": [r[1] for r in res]}
    path = os.path.join(HERE, "c4_bench_sample.json.gz")
    with gzip.open(path, "wt") as fh:
        json.dump(payload, fh, separators=(",", ":"))
    print("wrote", path, len(idx), "trees;",
          sum(1 for m in full_max if not m < LIM), "leave the asm range at 2^20")


if __name__ == "__main__":
    main()
