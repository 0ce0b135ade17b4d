#!/usr/bin/env python3
"""Price cheaper fp64 sin/cos variants against every fp64 golden (VERDICT r4
Next #1), on the CPU.

The product's sin/cos (gpeval.hip gp_trig, gen_asm.py trig_ops: 21 fp64
operations per call, near-correctly rounded) is modelled bit for bit by
scripts/trig_variants.c (flags 0); the variants drop terms from it.  Every
golden program is evaluated over its cases with numpy (add/sub/mul/div/neg
are IEEE and identical to the device's), sin/cos through the variant, and a
program whose sin/cos arguments reach the redo threshold (or are not finite)
is re-evaluated with glibc's sin/cos, as the product's redo pass does.  The
MSE (math.fsum of d*d, then / n) is compared with the reference's value.

Measurement only: not used by the product or the tests.

usage: python scripts/trig_sweep.py [--variants 0,1,2,...] [--thr 40,30,20]
       [--fixtures c4_bench_sample,...] [--out profiles/r05_trig_sweep.jsonl]
"""
import argparse
import ctypes
import gzip
import json
import math
import os
import subprocess
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from deap_amd import configs, datasets, gp            # noqa: E402
from deap_amd.flatten import Flattener               # noqa: E402

SO = "/tmp/trig_variants.so"
FLAG_NAMES = {1: "fold_rl", 2: "no_ae", 4: "deg1", 8: "no_low"}
# fp64 operations per call below 2^14 (the fast body)
OPS = {0: 21}


def n_ops(fl):
    n = 21
    if fl & 1:
        n -= 1
    if fl & 2:
        n -= 2
    if fl & 4:
        n -= 2
    if fl & 8:
        n -= 2 if fl & 2 else 1        # (no Sl/Cl: no fma(cl, t, sl))
        if fl & 2:
            n -= 1                     # a + z*tails in one fma
    return n


def build():
    src = os.path.join(HERE, "trig_variants.c")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-march=native",
                               "-ffp-contract=off", "-shared", "-fPIC", "-o",
                               SO, src, "-lm"])


def _lp_fit(res, cols):
    """min over q of max_i |res_i - sum_k q_k cols_k[i]| by Lawson's
    iteratively reweighted least squares (columns and residual scaled)."""
    res = np.asarray(res, np.float64)
    rs = np.abs(res).max()
    A = np.stack([np.asarray(c, np.float64) for c in cols], 1)
    cs = np.abs(A).max(0)
    A = A / cs
    y = res / rs
    w = np.full(len(y), 1.0 / len(y))
    for _ in range(500):
        sw = np.sqrt(w)
        q = np.linalg.lstsq(A * sw[:, None], y * sw, rcond=None)[0]
        e = np.abs(y - A @ q)
        w = w * e
        w /= w.sum()
    return list(q * rs / cs), float(e.max() * rs)


def minimax_deg1():
    """Degree-1 Ps (both coefficients) and Pc1 (with -1/2 fixed), minimax
    for the error they leave in sin r (relative) and cos r (absolute) over
    |r| <= pi/512; returns (Ps0, Ps1, Pc1, err_sin, err_cos)."""
    import mpmath
    mpmath.mp.prec = 200
    c = mpmath.pi / 512
    rs = [c * (i + 1) / 400 for i in range(400)]
    T0, T1 = -mpmath.mpf(1) / 6, mpmath.mpf(1) / 120
    # sin r = r + r^3 (P0 + P1 z): error / sin r
    res, c0, c1 = [], [], []
    for r in rs:
        z = r * r
        w = r ** 3 / mpmath.sin(r)
        f = (mpmath.sin(r) - r) / r ** 3
        res.append(float(w * (f - T0 - T1 * z)))
        c0.append(float(w))
        c1.append(float(w * z))
    (q0, q1), es = _lp_fit(res, [c0, c1])
    ps0 = float(T0 + mpmath.mpf(q0))
    ps1 = float(T1 + mpmath.mpf(q1))
    # cos r = 1 - z/2 + z^2 Pc1: absolute error
    U = mpmath.mpf(1) / 24
    res, c0 = [], []
    for r in rs:
        z = r * r
        g = ((mpmath.cos(r) - 1) / z + mpmath.mpf(1) / 2) / z
        res.append(float(z * z * (g - U)))
        c0.append(float(z * z))
    (q,), ec = _lp_fit(res, [c0])
    return ps0, ps1, float(U + mpmath.mpf(q)), es, ec


def load_consts(deg1):
    d = json.load(open(os.path.join(REPO, "deap_amd", "csrc",
                                    "trig_table.json")))
    h = float.fromhex
    tab = np.array([h(v) for row in d["table"] for v in row], np.float64)
    ps = [h(v) for v in d["Ps"]]
    pc = [h(v) for v in d["Pc"]]
    c = [h(d["INV"]), h(d["S1"]), -h(d["S2"])] + [h(v) for v in d["C"]] + \
        ps + pc[1:]
    c = np.array(c, np.float64)
    # the degree-1 coefficients (flag 4) follow
    c = np.concatenate([c, np.asarray(deg1 if deg1 else (ps[0], ps[1], pc[1]),
                                      np.float64)])
    return tab, c


class Lib(object):
    def __init__(self, deg1):
        self.lib = ctypes.CDLL(SO)
        tab, c = load_consts(deg1)
        self._keep = (tab, c)
        P = ctypes.c_void_p
        self.lib.tv_init.argtypes = [P, P]
        self.lib.tv_eval.argtypes = [ctypes.c_int, ctypes.c_int,
                                     ctypes.c_double, P, P, ctypes.c_int64, P]
        self.lib.tv_eval.restype = ctypes.c_int64
        self.lib.tv_libm.argtypes = [ctypes.c_int, P, P, ctypes.c_int64]
        self.lib.tv_init(tab.ctypes.data, c.ctypes.data)

    def trig(self, fl, cosine, lim, x):
        x = np.ascontiguousarray(x, np.float64)
        y = np.empty_like(x)
        m = np.zeros(1)
        if fl < 0:
            self.lib.tv_libm(cosine, x.ctypes.data, y.ctypes.data, x.size)
            return y, 0.0, 0
        nf = self.lib.tv_eval(fl, cosine, lim, x.ctypes.data, y.ctypes.data,
                              x.size, m.ctypes.data)
        return y, float(m[0]), int(nf)


class Skip(Exception):
    pass


def evaluate(tree, argidx, X, lib, fl, lim):
    """f over all cases (array or Python scalar); returns (f, max |arg|,
    non-finite args) with Python-number semantics for scalar subtrees."""
    st = []
    mx, nf = 0.0, 0
    for node in reversed(tree):
        if node.arity == 0:
            v = node.value
            st.append(X[argidx[v]] if isinstance(v, str) else v)
            continue
        args = [st.pop() for _ in range(node.arity)]
        name = node.name
        scalar = all(not isinstance(a, np.ndarray) for a in args)
        try:
            if name == "add":
                r = args[0] + args[1]
            elif name == "sub":
                r = args[0] - args[1]
            elif name == "mul":
                r = args[0] * args[1]
            elif name == "neg":
                r = -args[0]
            elif name == "protectedDiv":
                l, d = args
                if scalar:
                    try:
                        r = l / d
                    except ZeroDivisionError:
                        r = 1
                else:
                    with np.errstate(all="ignore"):
                        r = np.where(np.asarray(d) == 0, 1.0, np.divide(l, d))
            elif name in ("sin", "cos"):
                a = args[0]
                if scalar:
                    r = (math.sin if name == "sin" else math.cos)(a)
                else:
                    r, m, n = lib.trig(fl, name == "cos", lim, a)
                    mx = max(mx, m)
                    nf += n
            else:
                raise KeyError(name)
        except (OverflowError, ValueError):
            raise Skip()
        if isinstance(r, int) and abs(r) > 2 ** 53:
            raise Skip()                   # the exact-int pass's programs
        st.append(r)
    return st[0], mx, nf


def mse(f, T, n):
    d = np.broadcast_to(np.asarray(f, np.float64), (n,)).copy()
    with np.errstate(all="ignore"):
        for t in T:
            d = d - t
        sq = d * d
    if not np.isfinite(sq).all():
        return None
    return math.fsum(sq.tolist()) / n


FIXTURES = ["c1_symbreg", "c1_edge", "c4_symreg10", "c4_symreg10_1m",
            "c4_bench_sample", "c4_deep_core", "c4_evolved", "bench_pop"]


def fixture(name):
    """(pset, trees (strings), X, T, reference fitness list or None)."""
    from conftest import decode_fitness, load_golden
    if name == "bench_pop":
        # 2,000 trees of the headline population at 2^16 cases (reference
        # values: the same evaluation with glibc's sin/cos, fsum)
        pset = configs.pset_for("symreg10")
        pop = configs.population(pset, "half", 65536, 2024, 4, 8)
        idx = np.random.default_rng(5).choice(65536, 2000, replace=False)
        trees = [str(pop[i]) for i in sorted(idx.tolist())]
        X, y = datasets.symreg10_cases(2 ** 16, 2024)
        return "symreg10", trees, X, y, None
    if name == "c4_evolved":
        with gzip.open(os.path.join(REPO, "tests", "golden",
                                    "c4_evolved.json.gz"), "rt") as fh:
            g = json.load(fh)
        X, y = datasets.symreg10_cases(4096, 2024)
        return "symreg10", g["trees"], X, y, None
    g = load_golden(name)
    if g["pset"] == "symbreg":
        X, T = datasets.symbreg_points()
    else:
        d = g["data"]
        X, T = datasets.symreg10_cases(d.get("n", 2 ** 20), d.get("seed", 2024))
    ref = [None if e is not None else decode_fitness(f)
           for f, e in zip(g["fitness"], g["error"])]
    return g["pset"], g["trees"], X, T, ref


_CACHE = {}


def run_fixture(job):
    name, variants, thrs, deg1 = job
    pset_name, trees, X, T, ref = fixture(name)
    pset = configs.pset_for(pset_name)
    argidx = {a: i for i, a in enumerate(pset.arguments)}
    n = X.shape[1]
    lib = Lib(deg1)
    pts = [gp.PrimitiveTree.from_string(s, pset) for s in trees]
    depth = Flattener(pset).flatten(pts).depth
    if ref is None:                     # glibc evaluation (the reference)
        ref = []
        for t in pts:
            try:
                f, _, nf = evaluate(t, argidx, X, lib, -1, 0.0)
                ref.append(None if nf else mse(f, T, n))
            except Skip:
                ref.append(None)
    out = []
    for fl in variants:
        for tb in thrs:
            t0 = time.time()
            errs, redo, bad13, bad12, bitid, cnt = [], 0, 0, 0, 0, 0
            worst = None
            for i, t in enumerate(pts):
                exp = ref[i]
                if exp is None or not math.isfinite(exp):
                    continue
                lim = 2.0 ** (tb if depth[i] <= 5 else min(tb, 20))
                try:
                    f, mx, nf = evaluate(t, argidx, X, lib, fl, lim)
                except Skip:
                    continue
                if mx >= lim or nf:
                    redo += 1
                    f, _, _ = evaluate(t, argidx, X, lib, -1, 0.0)
                v = mse(f, T, n)
                if v is None:
                    continue
                cnt += 1
                rel = abs(v - exp) / abs(exp) if exp else abs(v)
                bitid += v == exp
                bad13 += rel > 1e-13
                bad12 += rel > 1e-12
                if worst is None or rel > worst[0]:
                    worst = (rel, trees[i][:160])
                errs.append(rel)
            out.append({"fixture": name, "flags": fl, "ops": n_ops(fl),
                        "thr_log2": tb, "programs": cnt, "redo": redo,
                        "bit_identical": bitid, "over_1e-13": bad13,
                        "over_1e-12": bad12,
                        "max_rel": worst[0] if worst else 0.0,
                        "worst_tree": worst[1] if worst else None,
                        "secs": round(time.time() - t0, 1)})
            print(json.dumps(out[-1]), flush=True)
    return out


def call_rates(deg1, variants, n=2_000_000):
    """Per-call disagreement with glibc on U(-50, 50) and U(-1, 1)."""
    lib = Lib(deg1)
    rng = np.random.default_rng(3)
    res = []
    for lo in (1.0, 50.0):
        x = rng.uniform(-lo, lo, n)
        for cos in (0, 1):
            g, _, _ = lib.trig(-1, cos, 0, x)
            for fl in variants:
                y, _, _ = lib.trig(fl, cos, 2.0 ** 40, x)
                d = np.count_nonzero(y != g)
                res.append({"range": lo, "fn": "cos" if cos else "sin",
                            "flags": fl, "differs_from_glibc": d / n})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,4,3,5,6,7,15")
    ap.add_argument("--thr", default="40")
    ap.add_argument("--fixtures", default=",".join(FIXTURES))
    ap.add_argument("--out", default="")
    ap.add_argument("--procs", type=int, default=6)
    a = ap.parse_args()
    build()
    variants = [int(v) for v in a.variants.split(",")]
    thrs = [int(v) for v in a.thr.split(",")]
    deg1 = minimax_deg1()
    print(json.dumps({"deg1_minimax": [float(v) for v in deg1],
                      "ops": {fl: n_ops(fl) for fl in variants}}))
    for r in call_rates(deg1[:3], variants, 400_000):
        print(json.dumps(r))
    jobs = [(f, variants, thrs, deg1[:3]) for f in a.fixtures.split(",")]
    with Pool(min(a.procs, len(jobs))) as p:
        res = [r for rr in p.map(run_fixture, jobs) for r in rr]
    if a.out:
        with open(a.out, "a") as fh:
            for r in res:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
