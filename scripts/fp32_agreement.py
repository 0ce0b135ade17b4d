#!/usr/bin/env python3
"""fp32 mode vs the reference's fp64 fitness on the committed goldens
(GPU): distribution of the relative MSE difference per tree, and hit-count
differences for the typed-GP set.  Prints one JSON line per golden set."""
import json
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import decode_fitness, load_golden  # noqa: E402
from deap_amd import configs, gp  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402


def main():
    for name in ("c1_symbreg", "c4_symreg10", "c4_symreg10_1m",
                 "np_symbreg", "c5_spambase"):
        g = load_golden(name)
        pset = configs.pset_for(g["pset"])
        spec = configs.spec_for(g["pset"], g["data"])
        ev = GPUEvaluator(pset, spec, device=0, precision="fp32")
        trees = [gp.PrimitiveTree.from_string(s, pset) for s in g["trees"]]
        got = ev.evaluate(trees)
        rel, exact, nonfin_mismatch, skipped = [], 0, 0, 0
        for res, fit, err in zip(got, g["fitness"], g["error"]):
            if err is not None or isinstance(res, BaseException):
                skipped += 1
                continue
            exp = decode_fitness(fit)
            val = res[0]
            if isinstance(exp, int):
                rel.append(abs(val - exp) / max(len(spec.X[0]), 1))
                exact += val == exp
                continue
            if not math.isfinite(exp) or not math.isfinite(val):
                nonfin_mismatch += not (exp == val or (math.isnan(exp) and
                                                       math.isnan(val)))
                continue
            rel.append(abs(val - exp) / max(abs(exp), 1e-300))
            exact += val == exp
        r = np.array(rel)
        q = {p: float(np.quantile(r, p)) for p in (0.5, 0.9, 0.99)} \
            if len(r) else {}
        print(json.dumps({
            "golden": name, "trees": len(trees), "compared": len(r),
            "skipped_errors": skipped, "nonfinite_mismatch": nonfin_mismatch,
            "median_rel": q.get(0.5), "p90_rel": q.get(0.9),
            "p99_rel": q.get(0.99), "max_rel": float(r.max()) if len(r) else
            None, "frac_within_1e-4": float((r <= 1e-4).mean()),
            "frac_within_1e-3": float((r <= 1e-3).mean()),
            "bit_equal": int(exact)}), flush=True)


if __name__ == "__main__":
    main()
