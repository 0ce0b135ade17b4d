#!/usr/bin/env python3
"""The host-flattener path of a BASELINE population (flatten once, then
run_batch = gpe_load_programs + gpe_run) with laps under GPE_DIAG.
Usage: GPE_DIAG=1 python scripts/hostflat_probe.py c3"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

from bench_configs import population  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    ev.evaluate(pop[:64])
    batch = ev.flatten(pop)
    for _ in range(4):
        t0 = time.perf_counter()
        ev.ctx.load_programs(batch)
        t1 = time.perf_counter()
        ev.ctx.run(spec.mode)
        t2 = time.perf_counter()
        print("%s load_programs %.2f ms, run %.2f ms" % (name, 1e3 * (t1 - t0), 1e3 * (t2 - t1)),
              file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
