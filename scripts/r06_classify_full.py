#!/usr/bin/env python3
"""Why each non-bit-identical tree of the full reference fixtures differs.

Reads the GPU fitness saved by scripts/r06_dump_full.py (gpurun_out/) and
the reference fixtures (tests/golden/c4_bench_full_2e16.json.gz,
c4_evolved_ref.json.gz).  For every tree whose GPU fitness is not the
reference's to the bit, the per-case errors d = f(x) - y are recomputed on
the host with the oracle (the reference's evaluation restated: gp.compile's
semantics, math.sin/cos) and the MSE formed three ways:

* ``ref``:  math.fsum(d ** 2) / n — the reference (d ** 2 is glibc's pow);
* ``mul``:  math.fsum(d * d) / n — the correctly rounded square, exact sum;
* ``dd``:   the squares d * d summed in double-double (TwoSum) in case
            order, hi + lo — the device's arithmetic, not its exact order.

Reason ``pow``: ref != mul and the GPU value is mul (pow(d, 2) misrounds
some d; the device squares with one multiply).  Reason ``sum``: ref == mul
(every square the same) — the device's double-double, not fsum's exact
rounding, decides the last bit.  Anything else is ``other`` (a device value
the host cannot explain: a bug).  Writes tests/golden/c4_full_notes.json,
which test_gpu.py reads: the trees allowed to differ, with their reason.

Usage: python scripts/r06_classify_full.py
"""
import base64
import gzip
import json
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import gp_ref                  # noqa: E402
from deap_amd import configs, datasets     # noqa: E402


def two_sum(a, b):
    s = a + b
    bb = s - a
    return s, (a - (s - bb)) + (b - bb)


def classify(strs, fit, gpu_by_mode, X, y):
    rows = list(zip(*X.tolist()))
    out = {}
    n_bad = 0
    for i in range(len(strs)):
        vals = [g[i] for g in gpu_by_mode.values()]
        if all(v == fit[i] or (math.isnan(v) and math.isnan(fit[i])) for v in vals):
            continue
        n_bad += 1
        func = gp_ref.compile_expr(strs[i], "symreg10")
        d = [func(*r) - t for r, t in zip(rows, y.tolist())]
        ref = math.fsum(v ** 2 for v in d) / len(d)
        mul = math.fsum(v * v for v in d) / len(d)
        hi = lo = 0.0
        for v in d:
            hi, e = two_sum(hi, v * v)
            lo += e
        dd = (hi + lo) / len(d)
        assert ref == fit[i], (i, ref, fit[i])
        if ref != mul and all(v == mul for v in vals):
            why = "pow"
        elif ref == mul:
            why = "sum"
        else:
            why = "other"
        out[str(i)] = {"why": why, "gpu": [float(v).hex() for v in vals],
                       "ref": ref.hex(), "mul": mul.hex(), "dd": dd.hex(),
                       "rel": max(abs(v - ref) / abs(ref) for v in vals)}
    return out, n_bad


def main():
    gout = os.path.join(REPO, "gpurun_out")
    notes = {}
    with gzip.open(os.path.join(REPO, "tests", "golden", "c4_bench_full_2e16.json.gz"), "rt") as fh:
        g = json.load(fh)
    fit = np.frombuffer(base64.b64decode(g["fitness_f64_b64"]), dtype="<f8")
    _, trees, _, _ = configs.headline_c4(65536, 128, 2024, 4, 8)
    strs = [str(t) for t in trees]
    X, y = datasets.symreg10_cases(2 ** 16, 2024)
    gpu = {m: np.load(os.path.join(gout, "r06_full_2e16_leaves%d.npy" % m)) for m in (1, 0)}
    notes["c4_bench_full_2e16"], n = classify(strs, fit, gpu, X, y[0])
    print("headline 2^16: %d trees differ from the reference in the last bits" % n)
    with gzip.open(os.path.join(REPO, "tests", "golden", "c4_evolved_ref.json.gz"), "rt") as fh:
        g = json.load(fh)
    fit = np.frombuffer(base64.b64decode(g["fitness_f64_b64"]), dtype="<f8")
    with gzip.open(os.path.join(REPO, "tests", "golden", "c4_evolved.json.gz"), "rt") as fh:
        strs = json.load(fh)["trees"]
    X, y = datasets.symreg10_cases(4096, 2024)
    gpu = {m: np.load(os.path.join(gout, "r06_evolved_leaves%d.npy" % m)) for m in (1, 0)}
    notes["c4_evolved_ref"], n = classify(strs, fit, gpu, X, y[0])
    print("evolved: %d trees differ" % n)
    for name, d in notes.items():
        whys = {}
        for v in d.values():
            whys[v["why"]] = whys.get(v["why"], 0) + 1
        print(name, whys, "max rel", max([v["rel"] for v in d.values()] or [0]))
    with open(os.path.join(REPO, "tests", "golden", "c4_full_notes.json"), "w") as fh:
        json.dump(notes, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
