#!/usr/bin/env python3
"""GPU fitness of every tree of the two reference fixtures
(tests/golden/c4_bench_full_2e16.json.gz, c4_evolved_ref.json.gz) through the
product path (GPUEvaluator, trig-leaf columns and inline sin/cos), saved as
raw float64 under gpurun_out/ for scripts/r06_classify_full.py."""
import gzip
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from deap_amd import configs, datasets, gp  # noqa: E402
from deap_amd.evaluator import GPUEvaluator, SymbRegMSE  # noqa: E402


def fits(res):
    return np.array([np.nan if isinstance(r, BaseException) else r[0] for r in res])


def main():
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    pset, trees, _, _ = configs.headline_c4(65536, 128, 2024, 4, 8)
    X, y = datasets.symreg10_cases(2 ** 16, 2024)
    for leaves in (True, False):
        ev = GPUEvaluator(pset, SymbRegMSE(np.ascontiguousarray(X), y), device=0,
                          trig_leaves=leaves)
        np.save(os.path.join(out, "r06_full_2e16_leaves%d.npy" % leaves),
                fits(ev.evaluate(trees)))
        ev.ctx.close()
    with gzip.open(os.path.join(REPO, "tests", "golden", "c4_evolved.json.gz"), "rt") as fh:
        strs = json.load(fh)["trees"]
    pset = configs.pset_for("symreg10")
    trees = [gp.PrimitiveTree.from_string(t, pset) for t in strs]
    X, y = datasets.symreg10_cases(4096, 2024)
    for leaves in (True, False):
        ev = GPUEvaluator(pset, SymbRegMSE(np.ascontiguousarray(X), y), device=0,
                          trig_leaves=leaves)
        np.save(os.path.join(out, "r06_evolved_leaves%d.npy" % leaves),
                fits(ev.evaluate(trees)))
        ev.ctx.close()
    print("saved")


if __name__ == "__main__":
    main()
