#!/usr/bin/env python3
"""cProfile of PopulationSharded.evaluate (C3 at 1M) at world 1 on one GPU:
the population-sharded path's host cost beside GPUEvaluator.evaluate.
Run with MASTER_ADDR=127.0.0.1 MASTER_PORT=... RANK=0 WORLD_SIZE=1."""
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench_configs import population  # noqa: E402
from deap_amd.distributed import PopulationSharded  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    pset, spec, pop = population("c3")
    ev = GPUEvaluator(pset, spec, device=0)
    ps = PopulationSharded(ev)
    ps.evaluate(pop[:64])
    for _ in range(3):
        t0 = time.perf_counter()
        ps.evaluate(pop)
        print("sharded evaluate %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
    for _ in range(2):
        t0 = time.perf_counter()
        ev.evaluate(pop)
        print("plain evaluate %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    ps.evaluate(pop)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(22)
    print(s.getvalue(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
