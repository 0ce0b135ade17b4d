#!/usr/bin/env python3
"""Device lowering alone (gpe_lower_programs) on a BASELINE population:
read_codes once, then N lowerings; prints wall ms per call.  Run under
rocprofv3 for lower_trees' kernel time and counters.
Usage: python scripts/lower_probe.py c3 [N]"""
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    r = ev.flattener.read_codes(pop)
    ev.ctx.set_lowering(*ev.flattener.lowering_tables())
    for i in range(reps):
        t0 = time.perf_counter()
        ev.ctx.lower_programs(*r)
        print("%s lower_programs %.2f ms" % (name, 1e3 * (time.perf_counter() - t0)),
              flush=True)


if __name__ == "__main__":
    main()
