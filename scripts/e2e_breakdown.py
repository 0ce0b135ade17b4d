#!/usr/bin/env python3
"""Where GPUEvaluator.evaluate's wall time goes on one population (C3 / C5
at their BASELINE sizes): host flattening, program upload + validation,
device run + D2H, fitness tuples.  Usage:
    DEAP_AMD_FLAT_TIMING=1 python scripts/e2e_breakdown.py c3 [threads...]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

import numpy as np  # noqa: E402

from bench_configs import population  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402


def main():
    name = sys.argv[1]
    pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    ev.evaluate(pop[:64])
    out = {"config": name, "pop": len(pop)}
    for rep in range(3):
        t0 = time.perf_counter()
        batch = ev.flatten(pop)
        t1 = time.perf_counter()
        ev.ctx.load_programs(batch)
        t2 = time.perf_counter()
        hi, lo, err, flags = ev.ctx.run(spec.mode)
        t3 = time.perf_counter()
        res = spec.finish_all(hi, lo, err, flags)
        t4 = time.perf_counter()
        # device lowering: node codes read on the host, words built on the GPU
        u0 = time.perf_counter()
        r = ev.flattener.read_codes(pop)
        u1 = time.perf_counter()
        if not ev._lowering_set:
            ev.ctx.set_lowering(*ev.flattener.lowering_tables())
            ev._lowering_set = True
        ev.ctx.lower_programs(*r)
        u2 = time.perf_counter()
        hi, lo, err, flags = ev.ctx.run(spec.mode)
        u3 = time.perf_counter()
        t5 = time.perf_counter()
        res2 = ev.evaluate(pop)
        t6 = time.perf_counter()
        assert len(res) == len(res2)
        out["rep%d" % rep] = {
            "read_codes_ms": round(1e3 * (u1 - u0), 1),
            "lower_ms": round(1e3 * (u2 - u1), 1),
            "run_after_lower_ms": round(1e3 * (u3 - u2), 1),
            "flatten_ms": round(1e3 * (t1 - t0), 1),
            "load_ms": round(1e3 * (t2 - t1), 1),
            "run_ms": round(1e3 * (t3 - t2), 1),
            "kernel_ms": round(ev.ctx.timing()["total_ms"], 2),
            "finish_ms": round(1e3 * (t4 - t3), 1),
            "evaluate_ms": round(1e3 * (t6 - t5), 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
