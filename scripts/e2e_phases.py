#!/usr/bin/env python3
"""Median wall time of each phase of a warm GPUEvaluator.evaluate at pop 1M
(C3 / C5): the host reads (read_codes), the lowering calls (lower_add /
lower_end), the batch bookkeeping, the run (plan + kernels + result copy) and
the fitness tuples — timers wrapped around the evaluator's own calls, no
profiler.  Usage: python scripts/e2e_phases.py c3 [reps]
"""
import os
import sys
import time
from collections import defaultdict

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

from bench_configs import population  # noqa: E402
from deap_amd import evaluator as evmod  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402

T = defaultdict(list)
CUR = defaultdict(float)


def wrap(obj, name, tag):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            CUR[tag] += time.perf_counter() - t0
    setattr(obj, name, g)


def main():
    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    ev.evaluate(pop[:64])
    wrap(ev.flattener, "read_codes", "read_codes")
    wrap(ev.ctx, "lower_add", "lower_add")
    wrap(ev.ctx, "lower_end", "lower_end")
    wrap(ev.ctx, "lower_begin", "lower_begin")
    wrap(ev, "_lowered_batch", "batch")
    wrap(ev, "prepare", "prepare")
    wrap(ev, "run_batch", "run")
    if hasattr(ev.spec, "finish_all"):
        wrap(ev.spec, "finish_all", "finish_all")
    wrap(evmod, "_tuples1", "tuples1")
    for i in range(reps + 2):
        CUR.clear()
        t0 = time.perf_counter()
        ev.evaluate(pop)
        tot = time.perf_counter() - t0
        if i < 2:
            continue
        T["total"].append(tot)
        for k, v in CUR.items():
            T[k].append(v)
    for k in ["total", "read_codes", "lower_begin", "lower_add", "lower_end",
              "batch", "prepare", "run", "finish_all", "tuples1"]:
        if k in T:
            v = np.array(T[k]) * 1e3
            print("%-12s median %7.3f ms  min %7.3f" % (k, np.median(v), v.min()))


if __name__ == "__main__":
    main()
