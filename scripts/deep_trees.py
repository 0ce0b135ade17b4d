#!/usr/bin/env python3
"""Throughput on larger trees (config 4's primitive set, heights up to 14):
how the population splits between the asm core (<= asmcore::D stack slots)
and the C++ kernels, and what each part costs.  One JSON line per height
range.

Usage: python scripts/deep_trees.py [--pop 8192] [--cases 262144]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from deap_amd import configs  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402


def run(ev, batch, reps=3):
    best = None
    for _ in range(reps):
        ev.run_batch(batch)
        t = ev.ctx.timing()["total_ms"]
        best = t if best is None else min(best, t)
    return best, ev.ctx.geometry()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=8192)
    ap.add_argument("--cases", type=int, default=1 << 18)
    ap.add_argument("--ranges", default="4-8,8-12,10-14")
    args = ap.parse_args()
    pset = configs.pset_for("symreg10")
    spec = configs.spec_for("symreg10", {"n": args.cases})
    ev = GPUEvaluator(pset, spec, device=0)
    for rg in args.ranges.split(","):
        lo, hi = map(int, rg.split("-"))
        pop = configs.population(pset, "half", args.pop, 7, lo, hi)
        batch = ev.flatten(pop)
        ms, geo = run(ev, batch)
        work = int(batch.length.sum()) * spec.n_cases
        D = int(ev.ctx.asm_depth()) if hasattr(ev.ctx, "asm_depth") else 5
        sel = np.nonzero(batch.depth > D)[0]
        out = {"heights": rg, "pop": len(pop), "cases": spec.n_cases,
               "mean_len": round(float(batch.length.mean()), 1),
               "depth_hist": np.bincount(batch.depth).tolist(),
               "ms": round(ms, 3), "gpops": round(work / ms / 1e6, 1),
               "geometry": geo}
        if len(sel):
            sub = ev.flatten([pop[i] for i in sel])
            ms2, _ = run(ev, sub)
            out["deep_share_nodes"] = round(
                float(batch.length[sel].sum() / batch.length.sum()), 4)
            out["deep_ms"] = round(ms2, 3)
            out["deep_gpops"] = round(
                int(sub.length.sum()) * spec.n_cases / ms2 / 1e6, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
