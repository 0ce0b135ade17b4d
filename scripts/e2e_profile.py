#!/usr/bin/env python3
"""cProfile of one warm GPUEvaluator.evaluate call on a BASELINE population
(c3 / c5 at pop 1M): where the host time of toolbox.map goes beside the
kernels.  Usage: python scripts/e2e_profile.py c3 [n_lines]
"""
import cProfile
import io
import pstats
import sys
import time
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

from bench_configs import population  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402


def main():
    name = sys.argv[1]
    n_lines = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    ev.evaluate(pop[:64])
    for _ in range(2):
        t0 = time.perf_counter()
        ev.evaluate(pop)
        print("%s evaluate %.1f ms" % (name, (time.perf_counter() - t0) * 1e3), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    ev.evaluate(pop)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(n_lines)
    print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
