#!/usr/bin/env python3
"""cProfile of warm GPUEvaluator.evaluate calls at pop 1M (C3 / C5): where
the Python side of evaluate spends its time.  Usage:
python scripts/e2e_cprofile.py c5 [reps]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

from bench_configs import population  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402


def main():
    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    ev.evaluate(pop[:64])
    ev.evaluate(pop)
    ev.evaluate(pop)
    t0 = time.perf_counter()
    for _ in range(reps):
        ev.evaluate(pop)
    print("plain: %.3f ms per evaluate" % ((time.perf_counter() - t0) * 1e3 / reps))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(reps):
        ev.evaluate(pop)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
