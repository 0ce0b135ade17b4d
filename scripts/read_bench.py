#!/usr/bin/env python3
"""Host read of a 1M population (Flattener.read_codes in 2^18 chunks): min and
median ms over 9 passes.  Usage: python3 scripts/read_bench.py c3|c5"""
import sys, time, os
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, 'scripts'))
from bench_configs import population
from deap_amd.flatten import Flattener
import numpy as np
pset, spec, pop = population(sys.argv[1])
fl = Flattener(pset)
print("trees", len(pop), "nodes", sum(len(t) for t in pop))
chunk=1<<18
ts=[]
for r in range(9):
    t0=time.perf_counter()
    for a in range(0, len(pop), chunk):
        fl.read_codes(pop, a, min(len(pop), a+chunk))
    ts.append(time.perf_counter()-t0)
print(chunk, "min %.2f med %.2f ms" % (min(ts)*1e3, np.median(ts)*1e3))
