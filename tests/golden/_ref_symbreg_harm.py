"""Run the reference's examples/gp/symbreg_harm.py main() (seed 318, HARM-GP
bloat control, gp.py:938-1133) and print its logbook as JSON.  Executed by
make_golden.py with PYTHONPATH pointing at the 2to3 scratch copy of the
reference; build container only."""
import contextlib
import io
import json
import os
import sys

copy = os.environ["PYTHONPATH"].split(os.pathsep)[0]
sys.path.insert(0, os.path.join(copy, "examples", "gp"))
import symbreg_harm  # noqa: E402  (reference example)

with contextlib.redirect_stdout(io.StringIO()):
    pop, log, hof = symbreg_harm.main()


def h(v):
    return float(v).hex()


rec = {"gen": log.select("gen"), "nevals": log.select("nevals")}
for chap in ("fitness", "size"):
    for f in ("avg", "std", "min", "max"):
        rec["%s_%s" % (chap, f)] = [h(v) for v in log.chapters[chap].select(f)]
rec["hof"] = str(hof[0])
rec["hof_fitness"] = h(hof[0].fitness.values[0])
print(json.dumps(rec))
