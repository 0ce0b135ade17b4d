#!/usr/bin/env python3
"""Per-handler cost of the fp64 asm core on the GPU: populations of one
synthetic expression shape (chains of one primitive) at 2^20 cases, kernel
time per node-case, next to the handler's instruction counts
(scripts/handler_mix.py's parser) — the cycles each handler takes against its
fp64 VALU issue bound (4 cycles per wave-instruction).

    python scripts/handler_cost.py [--pop N] [--cases N]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def chain(fn, depth, arg="ARG0", right=False, nv=10):
    """fn(fn(...fn(x)...)) for unary fn; for binary fn a left-deep
    (fn(fn(x0, x1), x2) ...) or right-deep (fn(x0, fn(x1, ...))) chain."""
    if fn in ("sin", "cos", "neg"):
        s = arg
        for _ in range(depth):
            s = "%s(%s)" % (fn, s)
        return s
    s = "ARG0"
    for i in range(1, depth + 1):
        v = "ARG%d" % (i % nv)
        s = "%s(%s, %s)" % (fn, v, s) if right else "%s(%s, %s)" % (fn, s, v)
    return s


def balanced(fn, depth, leaf=[0]):
    """A full binary fn-tree of the given depth over neg(ARGi) leaves (both
    children non-leaf: PUSH + fn on the stack slot)."""
    if depth == 0:
        leaf[0] += 1
        return "neg(ARG%d)" % (leaf[0] % 10)
    return "%s(%s, %s)" % (fn, balanced(fn, depth - 1), balanced(fn, depth - 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=16384)
    ap.add_argument("--cases", type=int, default=2 ** 20)
    ap.add_argument("--depth", type=int, default=32)
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
    shapes = [("sin", False), ("cos", False), ("neg", False),
              ("add", False), ("add", True), ("mul", False), ("mul", True),
              ("protectedDiv", False), ("protectedDiv", True),
              ("add", "bal"), ("mul", "bal")]
    out = []
    for fn, right in shapes:
        expr = (balanced(fn, 4) if right == "bal" else
                chain(fn, a.depth, right=right))
        tree = gp.PrimitiveTree.from_string(expr, pset)
        batch = fl.flatten([tree] * a.pop)
        ctx.load_programs(batch)
        ms = []
        for it in range(4):
            ctx.run(_lib.GPE_MODE_MSE)
            if it:
                ms.append(ctx.timing()["kernel_ms"])
        nodes = int(batch.length.sum())
        t = float(np.median(ms))
        ns = t * 1e6 / (nodes * a.cases)
        # cycles per wave-handler on one SIMD: 1024 SIMDs, 128 node-cases
        # per wave-handler (K = 2 cases x 64 lanes)
        cyc = t * 1e-3 * clock * 1e9 * 1024 / (nodes * a.cases / 128.0)
        rec = {"shape": "%s%s" % (fn, {True: "_right", False: "",
                                         "bal": "_balanced"}[right]),
               "nodes_per_tree": len(tree), "kernel_ms": round(t, 3),
               "gpops": round(nodes * a.cases / t / 1e6, 1),
               "simd_cycles_per_wave_node": round(cyc, 1),
               "geometry": ctx.geometry()}
        out.append(rec)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
