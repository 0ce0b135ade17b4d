#!/usr/bin/env python3
"""What stalls GPUEvaluator.evaluate at pop 1M: evaluate back to back, after
freeing a large numpy array, after a host flatten (freed / kept), after a
cProfile-free Python allocation burst.  Usage: python scripts/stall_probe.py c5
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
    name = sys.argv[1] if len(sys.argv) > 1 else "c5"
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    reps = 5
    # STALL_GC=freeze: gc.freeze() after setup (the population and
    # evaluator never scanned again); disable: no cyclic GC during the runs
    import gc
    mode = os.environ.get("STALL_GC", "")
    pset, spec, pop = population(name)
    ev = GPUEvaluator(pset, spec, device=0)
    ev.evaluate(pop[:64])
    out = {"config": name, "gc": mode,
           "malloc_env": {k: v for k, v in os.environ.items()
                          if k.startswith("MALLOC_")}}
    if mode == "freeze":
        gc.freeze()
    elif mode == "disable":
        gc.disable()

    def timed():
        t0 = time.perf_counter()
        ev.evaluate(pop)
        return round(1e3 * (time.perf_counter() - t0), 1)

    def want(k):
        return only is None or k in only

    out["back_to_back"] = [timed() for _ in range(reps)]
    if want("free"):
        r = []
        for _ in range(reps):
            a = np.ones(40_000_000)
            del a
            r.append(timed())
        out["after_free_320MB"] = r
    if want("flat"):
        r = []
        for _ in range(reps):
            b = ev.flatten(pop)
            del b
            r.append(timed())
        out["after_flatten_freed"] = r
        r = []
        keep = []
        for _ in range(reps):
            keep.append(ev.flatten(pop))
            r.append(timed())
        del keep
        out["after_flatten_kept"] = r
    if want("burst"):
        r = []
        for _ in range(reps):
            lst = [[i] for i in range(2_000_000)]
            del lst
            r.append(timed())
        out["after_pyobj_burst"] = r
    if want("sleep"):
        r = []
        for _ in range(reps):
            time.sleep(0.2)
            r.append(timed())
        out["after_sleep_200ms"] = r
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
