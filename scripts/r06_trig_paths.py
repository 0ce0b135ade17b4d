#!/usr/bin/env python3
"""Which glibc range blocks the exact core's sin/cos handlers run, per wave.

The exact core (gen_asm.py glibc_seq3) runs each of glibc's range blocks for
a chain of 64 cases whenever any of its lanes needs it (a wave-uniform skip
over both chains K = 2, then one block per chain under its lane mask).  This
script evaluates a sample of the headline population (numpy, sin/cos from
the host libm) on the first tiles of bench.py's cases, collects every
sin/cos call's 128 arguments per (node, tile), and counts how often each
block runs — the handler's dynamic instruction mix, priced with the static
counts of the generated handler.

Usage: python scripts/r06_trig_paths.py [trees=2048] [tiles=64]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(1, os.path.join(REPO, "tests", "golden"))

from deap_amd import gp as cgp  # noqa: E402
import _bench_sample as bs      # noqa: E402

LO_D, LO_E, LO_R = 0.855469, 2.426265, 105414350.0


def hi_le(x, h):
    """glibc's k < h test on the high word: |x| < the double (h << 32)."""
    return np.abs(x) < np.frombuffer(np.uint64(h << 32).tobytes(), "<f8")[0]


def collect(tree, X):
    calls = []

    def ev(i):
        node = tree[i]
        if isinstance(node, cgp.Terminal):
            v = node.value
            if isinstance(v, str):
                return X[int(v[3:])], i + 1
            return np.full(X.shape[1], float(v)), i + 1
        vals, j = [], i + 1
        for _ in range(node.arity):
            v, j = ev(j)
            vals.append(v)
        n = node.name
        with np.errstate(all="ignore"):
            if n == "add":
                return vals[0] + vals[1], j
            if n == "sub":
                return vals[0] - vals[1], j
            if n == "mul":
                return vals[0] * vals[1], j
            if n == "protectedDiv":
                z = vals[1] == 0
                return np.where(z, 1.0, vals[0] / np.where(z, 1.0, vals[1])), j
            if n == "neg":
                return -vals[0], j
            calls.append((n, vals[0]))
            return (np.sin if n == "sin" else np.cos)(vals[0]), j
    ev(0)
    return calls


def classify(kind, x):
    """Per chain (x shaped [tiles, 2, 64]): which blocks have lanes."""
    ax = np.abs(x)
    fin = np.isfinite(x)
    d = hi_le(x, 0x400368fd) & ~hi_le(x, 0x3feb6000)
    e = hi_le(x, 0x419921fb) & ~hi_le(x, 0x400368fd)
    r = fin & ~hi_le(x, 0x419921fb)
    # quadrant parity after the range step (do_cos lanes): sin: d lanes and
    # e/r lanes with odd n; cos: lanes outside d with ... (approximated by
    # the reduced quadrant of x * 2/pi)
    n = np.rint(x * (2 / np.pi)).astype(np.int64, copy=False) \
        if np.isfinite(x).all() else np.zeros(x.shape, np.int64)
    small = ~hi_le(x, 0x3feb6000) == False  # noqa: E712  |x| < 0.855469
    if kind == "sin":
        docos = d | ((e | r) & (n % 2 == 1))
    else:
        docos = small | ((e | r) & (n % 2 == 0))
    dosin = fin & ~docos
    # reduced |a| for the Taylor test (do_sin lanes)
    red = np.where(small, ax, np.abs(ax - np.abs(n) * (np.pi / 2)))
    red = np.where(d, np.abs(np.pi / 2 - ax), red)
    taylor = dosin & (red < 0.126)
    return {"d": d.any(-1), "e": e.any(-1), "r": r.any(-1),
            "bc": docos.any(-1), "bs": dosin.any(-1), "t": taylor.any(-1)}


def main():
    n_trees = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    tiles = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    pop = bs.bench_population()
    X = bs.bench_data()[:, :tiles * 128]
    idx = np.random.default_rng(6).choice(len(pop), n_trees, replace=False)
    tot = {k: np.zeros(2) for k in ("d", "e", "r", "bc", "bs", "t")}
    wave = {k: 0 for k in tot}
    calls = 0
    for i in idx.tolist():
        for kind, x in collect(pop[i], X):
            c = classify(kind, x.reshape(tiles, 2, 64))
            calls += tiles
            for k, v in c.items():
                tot[k] += v.sum(0)
                wave[k] += int(v.any(-1).sum())
    print("sin/cos wave-calls: %d (trees %d, tiles %d)" % (calls, n_trees, tiles))
    for k in tot:
        print("%-3s wave-uniform %.3f   per chain %.3f %.3f"
              % (k, wave[k] / calls, tot[k][0] / calls, tot[k][1] / calls))


if __name__ == "__main__":
    main()
