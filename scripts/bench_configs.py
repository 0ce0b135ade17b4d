#!/usr/bin/env python3
"""Per-configuration throughput of one population evaluation (GPU), beside
bench.py's C4 headline: BASELINE.json configs 1, 2, 3, 5 plus the numpy and
ADF examples, at their stated sizes.  One JSON line per config:

* ``kernel_gpops``  node-evals x cases / device time of the evaluation
  kernels (HIP events on the context stream);
* ``device_gpops``  ... / wall time of ``evaluate``'s device calls
  (``device_ms``: device lowering, kernels, result copy);
* ``e2e_gpops``     ... / wall time of ``GPUEvaluator.evaluate`` (reading
  the trees, device, fitness tuples) — what ``toolbox.map`` costs;
* ``hostflat_flatten_ms`` / ``hostflat_device_ms``: the host-flattener path
  (``evaluate`` falls back to it for trees the device lowering declines):
  flattening, then program upload + kernels + D2H.

Usage: python scripts/bench_configs.py [--only c3,c5] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from deap_amd import configs, gp, tools  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402

# name -> (pset, spec data, generator, pop, min, max, seed)
CONFIGS = {
    "c1": ("symbreg", {}, "half", 300, 1, 2, 318),
    "c2": ("mux11", {}, "full", 40000, 2, 4, 201),
    "c3": ("parity6", {}, "full", 1000000, 3, 5, 301),
    "c5": ("spambase", {"n": 4601, "seed": 5}, "half", 1000000, 1, 2, 501),
    # the reference's own rows (examples/gp/spambase.csv, tests/golden)
    "c5_real": ("spambase", {"kind": "spambase_csv", "file": "spambase.csv.gz"},
                "half", 1000000, 1, 2, 511),
    "c5_deep": ("spambase", {"n": 4601, "seed": 5}, "half", 100000, 2, 6,
                502),
    "np": ("symbreg_numpy", {}, "half", 300, 1, 2, 318),
}


def population(name):
    pset_name, data, gen, n, lo, hi, seed = CONFIGS[name]
    pset = configs.pset_for(pset_name)
    return pset, configs.spec_for(pset_name, data), \
        configs.population(pset, gen, n, seed, lo, hi)


def adf_population(n, seed):
    import random
    psets = configs.pset_for("adf_symbreg")
    main_set, a0, a1, a2 = psets
    random.seed(seed)
    pop = []
    for _ in range(n):
        pop.append([gp.PrimitiveTree(gp.genHalfAndHalf(main_set, 1, 2)),
                    gp.PrimitiveTree(gp.genFull(a0, 1, 2)),
                    gp.PrimitiveTree(gp.genFull(a1, 1, 2)),
                    gp.PrimitiveTree(gp.genFull(a2, 1, 2))])
    return psets, configs.spec_for("adf_symbreg"), pop


def measure(name, reps, keep=False):
    """keep: also return the population and the last evaluation's results."""
    if name == "adf":
        pset, spec, pop = adf_population(100, 1024)
    else:
        pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    # warm up at full size: the first call of a population size allocates
    # the device buffers and pinned staging (in a GA every later generation
    # reuses them)
    ev.evaluate(pop)
    e2e, dev, kern, flat, hdev = [], [], [], [], []
    batch = None
    res = None
    for _ in range(reps):
        # (the previous evaluation's 1M result tuples are freed outside the
        # timed region: in a GA their fitness objects outlive the call)
        res = None
        d0 = ev.stats["device_s"]
        t0 = time.perf_counter()
        res = ev.evaluate(pop)
        e2e.append(time.perf_counter() - t0)
        # the evaluate's device calls (lowering + run + result copy)
        dev.append(ev.stats["device_s"] - d0)
        kern.append(ev.ctx.timing()["total_ms"] / 1e3)
    # the host-flattener legs after the evaluate loop: freeing a host-flattened
    # batch (millions of small Python objects) just before an evaluate stalled
    # that evaluate's first GPU operation by 10-30 ms on the box
    for _ in range(reps):
        batch = None
        t0 = time.perf_counter()
        batch = ev.flatten(pop)
        flat.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        ev.run_batch(batch)
        hdev.append(time.perf_counter() - t0)
    work = int(batch.length.sum()) * spec.n_cases
    n_err = sum(isinstance(r, BaseException) for r in res)
    rec = {"config": name, "pop": len(pop), "cases": spec.n_cases,
            "nodes": int(batch.length.sum()), "node_evals": work,
            "kernel_ms": round(1e3 * min(kern), 3),
            # device_ms: evaluate's device calls (gpe_lower_programs + gpe_run
            # with the result copy); hostflat_*: the host-flattener path
            # (flatten, then gpe_load_programs + gpe_run)
            "device_ms": round(1e3 * min(dev), 3),
            "e2e_ms": round(1e3 * min(e2e), 3),
            "e2e_ms_all": [round(1e3 * x, 2) for x in e2e],
            "hostflat_flatten_ms": round(1e3 * min(flat), 3),
            "hostflat_device_ms": round(1e3 * min(hdev), 3),
            "kernel_gpops": round(work / min(kern) / 1e9, 2),
            "device_gpops": round(work / min(dev) / 1e9, 2),
            "e2e_gpops": round(work / min(e2e) / 1e9, 2),
            "geometry": ev.ctx.geometry(), "errors": n_err}
    return (rec, pop, res) if keep else rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c1,c2,c3,c5,c5_deep,np,adf")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    for name in args.only.split(","):
        print(json.dumps(measure(name, args.reps)), flush=True)


if __name__ == "__main__":
    main()
