#!/usr/bin/env python3
"""Per-node and per-program cost of the fp64 asm core: chains of one
primitive at several lengths (one population per shape, every tree the same)
at 2^20 cases.  Kernel time per program-tile = a + b * nodes: b is the
handler's cost, a what each program costs beside its nodes (the loop's first
window load, the END epilogue, RELOADs are in b's steps every 15 words).
SIMD cycles per wave-node as scripts/handler_cost.py.

    python scripts/overhead_probe.py [--pop N] [--cases N]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))
from handler_cost import chain  # noqa: E402


def pushv_shape(n, nv=10):
    """add(neg(x0), add(neg(x1), ...)): every level a PUSHV + NEG + ADD_S."""
    s = "neg(ARG%d)" % (n % nv)
    for i in range(n):
        s = "add(neg(ARG%d), %s)" % (i % nv, s)
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=16384)
    ap.add_argument("--cases", type=int, default=2 ** 20)
    ap.add_argument("--shapes", default="neg,add,pushv,sin")
    ap.add_argument("--lengths", default="8,16,32,64,128")
    a = ap.parse_args()
    from deap_amd import _lib, configs, datasets, gp
    from deap_amd.flatten import Flattener
    pset = configs.pset_for("symreg10")
    rng = np.random.default_rng(7)
    X = np.ascontiguousarray(rng.uniform(-1.0, 1.0, size=(a.cases, 10)).T)
    y = datasets.unwrapped_ball_py(X)[None, :]
    ctx = _lib.Context(0)
    clock = ctx.device_info()["clock_khz"] / 1e6
    ctx.set_cases(_lib.GPE_MACHINE_F, X, y)
    fl = Flattener(pset)
    for shape in a.shapes.split(","):
        pts = []
        for L in map(int, a.lengths.split(",")):
            expr = pushv_shape(L // 3) if shape == "pushv" else chain(shape, L)
            tree = gp.PrimitiveTree.from_string(expr, pset)
            batch = fl.flatten([tree] * a.pop)
            ctx.load_programs(batch)
            ms = []
            for it in range(4):
                ctx.run(_lib.GPE_MODE_MSE)
                if it:
                    ms.append(ctx.timing()["kernel_ms"])
            t = float(np.median(ms))
            nodes = len(tree)
            words = int(batch.offsets[1] - batch.offsets[0])
            # SIMD cycles per wave-program-tile (K = 2: 128 cases per tile)
            wpt = a.pop * a.cases / 128.0
            cyc_prog = t * 1e-3 * clock * 1e9 * 1024 / wpt
            rec = {"shape": shape, "nodes": nodes, "words": words,
                   "kernel_ms": round(t, 3),
                   "simd_cycles_per_wave_program_tile": round(cyc_prog, 1),
                   "simd_cycles_per_wave_node": round(cyc_prog / nodes, 2)}
            pts.append((nodes, cyc_prog))
            print(json.dumps(rec), flush=True)
        n, c = np.array(pts, dtype=float).T
        b, a0 = np.polyfit(n, c, 1)
        print(json.dumps({"shape": shape, "fit_per_node": round(b, 2),
                          "fit_per_program_tile": round(a0, 1)}), flush=True)


if __name__ == "__main__":
    main()
