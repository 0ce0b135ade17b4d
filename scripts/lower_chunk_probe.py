#!/usr/bin/env python3
"""Chunked device lowering (gpe_lower_begin/add/end) of a BASELINE
population, each call timed on the host; the one-call path beside it.
Usage: python scripts/lower_chunk_probe.py c3 [chunk]"""
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
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 18
    pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    ev.evaluate(pop[:64])
    ev._set_lowering()
    fl, ctx, n = ev.flattener, ev.ctx, len(pop)
    for rep in range(4):
        t = [time.perf_counter()]
        ctx.lower_begin(n)
        t.append(time.perf_counter())
        for a in range(0, n, chunk):
            r = fl.read_codes(pop, a, min(n, a + chunk))
            t.append(time.perf_counter())
            ctx.lower_add(*r)
            t.append(time.perf_counter())
        ctx.lower_end()
        t.append(time.perf_counter())
        d = [round(1e3 * (y - x), 2) for x, y in zip(t, t[1:])]
        print("chunked total %.2f ms: begin %s, (read, add)... %s, end %s"
              % (1e3 * (t[-1] - t[0]), d[0], d[1:-1], d[-1]), flush=True)
        t0 = time.perf_counter()
        r = fl.read_codes(pop)
        t1 = time.perf_counter()
        ctx.lower_programs(*r)
        t2 = time.perf_counter()
        print("one call total %.2f ms: read %.2f, lower %.2f" % (1e3 * (t2 - t0), 1e3 * (t1 - t0),
                                                              1e3 * (t2 - t1)), flush=True)


if __name__ == "__main__":
    main()
