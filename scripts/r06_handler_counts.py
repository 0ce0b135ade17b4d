#!/usr/bin/env python3
"""Dynamic instruction counts of the exact sin/cos handlers on the headline
population's own arguments (tests/asm_emu.py on the CPU).

The sin/cos calls of a sample of bench trees on the first tiles of bench.py's
cases (scripts/r06_trig_paths.py collect()) are run wave by wave (128
arguments: chain k = cases 64k..64k+63 of the tile) through each generated
handler; the executed VALU (of them fp64), SALU and LDS instructions are
averaged per call, and every result is checked bit for bit against the host
libm.  Usage:

    python scripts/r06_handler_counts.py [trees=96] [tiles=4] [dir=suffix ...]

with core directories as ``path:suffix`` (default: the tree's own
deap_amd/csrc:_exact); e.g. a glibc_seq3 core generated into /tmp/seq3 with
GEN_ASM_GLIBC4=0: ``/tmp/seq3:_exact``.
"""
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(1, REPO)
sys.path.insert(2, os.path.join(REPO, "scripts"))
sys.path.insert(3, os.path.join(REPO, "tests", "golden"))

import asm_emu                  # noqa: E402
import r06_trig_paths as tp     # noqa: E402
import _bench_sample as bs      # noqa: E402


def main():
    n_trees = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    tiles = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    cores = sys.argv[3:] or ["%s:_exact" % asm_emu.CSRC]
    pop = bs.bench_population()
    X = bs.bench_data()[:, :tiles * 128]
    idx = np.random.default_rng(6).choice(len(pop), n_trees, replace=False)
    calls = []
    for i in idx.tolist():
        for kind, x in tp.collect(pop[i], X):
            for t in range(tiles):
                calls.append((kind, np.ascontiguousarray(x[t * 128:(t + 1) * 128])))
    print("%d wave-calls (%d trees x %d tiles)" % (len(calls), n_trees, tiles))
    for spec in cores:
        path, suffix = spec.rsplit(":", 1)
        lines = {w: asm_emu.handler_lines(w, suffix, path) for w in ("SIN", "COS")}
        counts, bad = {}, 0
        for kind, x in calls:
            if not np.isfinite(x).all():
                continue
            w = kind.upper()
            y, _ = asm_emu.run_handler(w, x, suffix, lines[w], path, counts)
            f = math.sin if kind == "sin" else math.cos
            ref = np.array([f(v) for v in x.tolist()])
            bad += int((y.view(np.uint64) != ref.view(np.uint64)).sum())
        n = len(calls)
        print("%-40s per call: VALU %.1f (fp64 %.1f)  SALU %.1f  LDS %.1f  | "
              "results not the host libm's: %d"
              % (spec, counts.get("valu", 0) / n, counts.get("valu_f64", 0) / n,
                 counts.get("salu", 0) / n, counts.get("lds", 0) / n, bad))


if __name__ == "__main__":
    main()
