#!/usr/bin/env python3
"""Reference fitness of EVERY tree of bench.py's headline population, and of
every tree of the evolved C4 populations.

1. ``c4_bench_full_2e16.json.gz``: all 65,536 headline trees
   (``configs.population(pset, "half", 65536, 2024, 4, 8)``) at the first
   2**16 of bench.py's cases (X ~ U(-1, 1) from ``default_rng(2024)``,
   variable-planar, columns 0..65535).
2. ``c4_evolved_ref.json.gz``: all 4,096 trees of ``c4_evolved.json.gz``
   at ``datasets.symreg10_cases(4096, 2024)``.

Both are evaluated by the REFERENCE: its ``gp.compile``
(``deap/gp.py:462-487``) and the ``examples/gp/symbreg.py:60-61`` loop shape
(``math.fsum((func(*x) - y)**2 ...) / len(points)``), with the target from
its ``deap/benchmarks/gp.py:60-72`` ``unwrapped_ball`` (checked bit-equal to
``datasets.unwrapped_ball_py``), one tree per task on a fork pool — the
evaluation ``deap/algorithms.py:172`` runs for every invalid individual.

The fixtures hold data only: fitness as the raw little-endian float64 bits
(base64; nan where the reference raised), the exception type names by
index, the sha256 of the tree strings in order (the GPU test regenerates the
population and checks it) and the data hashes.

Run in the build container only (needs the 2to3 copy of the reference,
``make_oracle_copy.sh``; about 40 min on 8 cores for part 1):
``python3 tests/golden/_bench_full.py [bench|evolved|all]``.  Finished chunks
are cached under ``/tmp/bench_full_parts`` so an interrupted run resumes.
"""
import base64
import gzip
import hashlib
import json
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ORACLE_COPY = os.environ.get("DEAP_ORACLE_COPY", "/tmp/deap_oracle")
PARTS = os.environ.get("BENCH_FULL_PARTS", "/tmp/bench_full_parts")
sys.path.insert(0, HERE)
sys.path.insert(1, REPO)

import _bench_sample as bs          # noqa: E402  (bench_data, bench_population)

N_CASES = 2 ** 16
CHUNK = 256
_G = {}


def _eval_chunk(args):
    """Reference fitness of trees [lo, hi) of _G["strs"] on _G's rows."""
    tag, lo, hi = args
    path = os.path.join(PARTS, "%s_%06d_%06d.json" % (tag, lo, hi))
    if os.path.exists(path):
        with open(path) as fh:
            return json.load(fh)
    sys.path.insert(0, ORACLE_COPY)
    import math
    from deap import gp  # the reference (2to3 copy)
    import make_golden
    pset = make_golden.arith_pset(10, False)
    rows, ys = _G["rows"], _G["y"]
    out = []
    for s in _G["strs"][lo:hi]:
        def mse():
            func = gp.compile(s, pset)
            return math.fsum((func(*x) - y) ** 2 for x, y in zip(rows, ys)) \
                / len(rows)
        val, err = make_golden.run(mse)
        out.append((make_golden.enc(val), err))
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        json.dump(out, fh)
    os.replace(tmp, path)
    return out


def _ref_target(X):
    sys.path.insert(0, ORACLE_COPY)
    from deap.benchmarks import gp as bgp   # reference benchmarks/gp.py
    from deap_amd import datasets
    rows = list(zip(*[col.tolist() for col in X]))
    y_ref = np.array([bgp.unwrapped_ball(r) for r in rows])
    assert datasets.unwrapped_ball_py(X).tobytes() == y_ref.tobytes()
    return rows, y_ref


def _run(tag, strs, X, workers):
    rows, y_ref = _ref_target(X)
    _G["strs"], _G["rows"], _G["y"] = strs, rows, y_ref.tolist()
    os.makedirs(PARTS, exist_ok=True)
    chunks = [(tag, lo, min(len(strs), lo + CHUNK))
              for lo in range(0, len(strs), CHUNK)]
    res = []
    with mp.get_context("fork").Pool(workers) as pool:
        for k, part in enumerate(pool.imap(_eval_chunk, chunks)):
            res.extend(part)
            if k % 16 == 0:
                print("%s: %d / %d trees" % (tag, len(res), len(strs)),
                      flush=True)
    fit = np.array([float.fromhex(v) if isinstance(v, str) else
                    (float(v) if v is not None else np.nan)
                    for v, _ in res], dtype="<f8")
    errors = {str(i): e for i, (_, e) in enumerate(res) if e is not None}
    return y_ref, fit, errors


def _payload(strs, X, y_ref, fit, errors, extra):
    p = {"pset": "symreg10",
         "data": {"n": X.shape[1],
                  "sha256_X": hashlib.sha256(X.tobytes()).hexdigest(),
                  "sha256_y_ref": hashlib.sha256(y_ref.tobytes()).hexdigest(),
                  "y": "reference deap/benchmarks/gp.py:60-72 unwrapped_ball"},
         "n_trees": len(strs),
         "sha256_trees": hashlib.sha256(
             "\n".join(strs).encode()).hexdigest(),
         "fitness_f64_b64": base64.b64encode(fit.tobytes()).decode(),
         "error": errors}
    p.update(extra)
    return p


def _dump(name, payload):
    path = os.path.join(HERE, name)
    with gzip.open(path, "wt") as fh:
        json.dump(payload, fh, separators=(",", ":"))
    print("wrote", path, payload["n_trees"], "trees,",
          len(payload["error"]), "errors")


def bench(workers):
    strs = [str(t) for t in bs.bench_population()]
    X = np.ascontiguousarray(bs.bench_data()[:, :N_CASES])
    y_ref, fit, errors = _run("bench", strs, X, workers)
    _dump("c4_bench_full_2e16.json.gz", _payload(
        strs, X, y_ref, fit, errors,
        {"population": {"generator": "half", "n": bs.POP, "seed": bs.SEED,
                        "min": bs.MIN_D, "max": bs.MAX_D},
         "cases": {"kind": "bench", "seed": bs.SEED, "of": bs.CASES,
                   "first": N_CASES}}))


def evolved(workers):
    from deap_amd import datasets
    with gzip.open(os.path.join(HERE, "c4_evolved.json.gz"), "rt") as fh:
        strs = json.load(fh)["trees"]
    X, _ = datasets.symreg10_cases(4096, 2024)
    X = np.ascontiguousarray(X)
    y_ref, fit, errors = _run("evolved", strs, X, workers)
    _dump("c4_evolved_ref.json.gz", _payload(
        strs, X, y_ref, fit, errors,
        {"cases": {"kind": "symreg10_cases", "n": 4096, "seed": 2024}}))


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    workers = int(os.environ.get("BENCH_FULL_WORKERS", "8"))
    if what in ("evolved", "all"):
        evolved(workers)
    if what in ("bench", "all"):
        bench(workers)
