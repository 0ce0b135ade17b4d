"""Relative SSE difference GPU vs reference goldens for config-4 trees,
split by whether the tree contains sin/cos."""
import json
import math
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import decode_fitness, load_golden
from deap_amd import configs, gp
from deap_amd.evaluator import GPUEvaluator

out = {}
for name in ("c4_symreg10", "c4_symreg10_1m", "c1_symbreg"):
    g = load_golden(name)
    pset = configs.pset_for(g["pset"])
    ev = GPUEvaluator(pset, configs.spec_for(g["pset"], g["data"]), device=0)
    trees = [gp.PrimitiveTree.from_string(s, pset) for s in g["trees"]]
    got = ev.evaluate(trees)
    rel_trig, rel_plain = [], []
    for s, r, f in zip(g["trees"], got, g["fitness"]):
        if f is None or isinstance(r, BaseException):
            continue
        e = decode_fitness(f)
        v = r[0]
        if not math.isfinite(e) or e == 0:
            continue
        rel = abs(v - e) / abs(e)
        (rel_trig if ("sin(" in s or "cos(" in s) else rel_plain).append(rel)
    def st(a):
        a = np.array(a) if a else np.zeros(1)
        return {"n": len(a), "max": float(a.max()),
                "p99": float(np.quantile(a, 0.99)),
                "frac_gt_1e-12": float((a > 1e-12).mean()),
                "frac_exact": float((a == 0).mean())}
    out[name] = {"trig": st(rel_trig), "no_trig": st(rel_plain)}
print(json.dumps(out, indent=1))
