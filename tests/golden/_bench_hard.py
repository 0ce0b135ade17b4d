#!/usr/bin/env python3
"""Golden fitness for the bench population's ill-conditioned programs.

bench.py's headline population (``configs.population(pset, "half", 65536,
2024, 4, 8)``, X ~ U(-1, 1) from ``default_rng(2024)``, 2**20 cases) holds
programs whose MSE moves by more than 1e-12 relative when a few of their
sin/cos values change in the last bit — typically a protectedDiv whose
denominator nearly cancels at one case that then dominates the sum.  Any
sin/cos that is not glibc's to the bit (the round-1..4 table sin/cos, which
differs from glibc wherever glibc misrounds, ~0.2 % of calls) misses the
north star's 1e-12 on them.

1. Scan: every tree at the first 2**16 cases, evaluated twice with numpy —
   sin/cos from glibc (the host libm: the reference's math.sin/cos) and
   from the table sin/cos model (scripts/trig_variants.c flags 0, programs
   with an argument past 2**40 re-run with glibc as the old redo pass did)
   — keeping trees whose two MSEs differ by more than 1e-12 relative.
2. Reference: those trees (at most 32) evaluated by the REFERENCE at all
   2**20 cases: its ``gp.compile`` (``deap/gp.py:462-487``) and the
   ``examples/gp/symbreg.py:60-61`` loop shape
   (``math.fsum((func(*x) - y)**2 ...) / len(points)``), the target from
   its ``deap/benchmarks/gp.py:60-72`` (as ``_bench_sample.py``).

Run in the build container only (needs the 2to3 copy of the reference,
``make_oracle_copy.sh``): ``python3 tests/golden/_bench_hard.py``.
Writes ``c4_bench_hard.json.gz``.
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
sys.path.insert(2, os.path.join(REPO, "scripts"))

import _bench_sample as bs          # noqa: E402  (bench_data, _ref_eval)

N_SCAN = 2 ** 16
N_KEEP = 32
_G = {}                 # the population and scan data, shared by fork


def _scan(args):
    lo, hi = args
    import trig_sweep as ts
    from deap_amd import configs, datasets
    pset = configs.pset_for("symreg10")
    pop, X, y = _G["pop"], _G["X"], _G["y"]
    lib = ts.Lib(None)
    argidx = {a: i for i, a in enumerate(pset.arguments)}
    out = []
    for i in range(lo, hi):
        try:
            fg, _, nf = ts.evaluate(pop[i], argidx, X, lib, -1, 0.0)
            ft, mx, nft = ts.evaluate(pop[i], argidx, X, lib, 0, 2.0 ** 40)
        except ts.Skip:
            continue
        if nf or nft or not mx < 2.0 ** 40:
            continue
        g, t = ts.mse(fg, y, N_SCAN), ts.mse(ft, y, N_SCAN)
        if g is None or t is None or g == 0:
            continue
        rel = abs(t - g) / abs(g)
        if rel > 1e-12:
            out.append((i, rel))
    return out


def main():
    import trig_sweep as ts
    ts.build()
    from deap_amd import datasets
    pop = bs.bench_population()
    strs = [str(t) for t in pop]
    _G["pop"] = pop
    _G["X"] = np.ascontiguousarray(bs.bench_data()[:, :N_SCAN])
    _G["y"] = datasets.unwrapped_ball_py(_G["X"])[None, :]
    chunks = [(lo, min(bs.POP, lo + 1024)) for lo in range(0, bs.POP, 1024)]
    with mp.get_context("fork").Pool(8) as pool:
        found = [r for part in pool.map(_scan, chunks) for r in part]
    found.sort(key=lambda r: -r[1])
    print("table sin/cos past 1e-12 at 2^16 cases: %d of %d trees"
          % (len(found), bs.POP))
    idx = sorted(i for i, _ in found[:N_KEEP])
    X = bs.bench_data()
    sys.path.insert(0, ORACLE_COPY)
    from deap.benchmarks import gp as bgp   # reference benchmarks/gp.py
    rows = list(zip(*[col.tolist() for col in X]))
    y_ref = np.array([bgp.unwrapped_ball(r) for r in rows])
    assert datasets.unwrapped_ball_py(X).tobytes() == y_ref.tobytes()
    bs._REF["rows"], bs._REF["y"] = rows, y_ref.tolist()
    with mp.get_context("fork").Pool(8) as pool:
        res = pool.map(bs._ref_eval, [strs[i] for i in idx], chunksize=1)
    payload = {
        "pset": "symreg10",
        "data": {"kind": "bench", "seed": bs.SEED, "n": bs.CASES,
                 "sha256_X": hashlib.sha256(X.tobytes()).hexdigest(),
                 "sha256_y_ref": hashlib.sha256(y_ref.tobytes()).hexdigest(),
                 "y": "reference deap/benchmarks/gp.py:60-72 unwrapped_ball"},
        "population": {"generator": "half", "n": bs.POP, "seed": bs.SEED,
                       "min": bs.MIN_D, "max": bs.MAX_D},
        "scan": {"cases": N_SCAN, "found": len(found),
                 "table_rel_at_scan": {str(i): r for i, r in found[:N_KEEP]}},
        "index": idx, "trees": [strs[i] for i in idx],
        "fitness": [r[0] for r in res], "error": [r[1] for r in res]}
    path = os.path.join(HERE, "c4_bench_hard.json.gz")
    with gzip.open(path, "wt") as fh:
        json.dump(payload, fh, separators=(",", ":"))
    print("wrote", path, len(idx), "trees")


if __name__ == "__main__":
    main()
