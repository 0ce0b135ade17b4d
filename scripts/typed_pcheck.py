#!/usr/bin/env python3
"""Typed core vs the C++ interpreter at several programs-per-wave settings
(GPE_TYPED_PMAX, read at context creation): first mismatching individual."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from deap_amd import configs  # noqa: E402
from deap_amd.evaluator import GPUEvaluator  # noqa: E402

pset = configs.pset_for("spambase")
spec = configs.spec_for("spambase", {"n": 4601, "seed": 5})
pop = configs.population(pset, "half", 60000, 77, 1, 4)
os.environ["GPE_TYPED_ASM"] = "0"
ev = GPUEvaluator(pset, spec, device=0)
ref = [r[0] for r in ev.evaluate(pop)]
ev.ctx.close()
os.environ["GPE_TYPED_ASM"] = "1"
for p in sys.argv[1:]:
    os.environ["GPE_TYPED_PMAX"] = p
    ev = GPUEvaluator(pset, spec, device=0)
    got = [r[0] for r in ev.evaluate(pop)]
    g = ev.ctx.geometry()
    bad = [i for i in range(len(pop)) if got[i] != ref[i]]
    print("P=%s geo P=%d groups=%d bad=%d first=%s" % (p, g["asm_typed_P"], g["asm_typed_groups"],
          len(bad), [(i, got[i], ref[i], str(pop[i])[:60]) for i in bad[:3]]), flush=True)
    ev.ctx.close()
