#!/usr/bin/env python3
"""Misround count of the table sin/cos (host twin of the kernels' gp_trig,
``_lib.host_math``) and of glibc (Python's math) against correctly rounded
results (mpmath, 200 bits), on CPU.  The asm cores and the C++ kernels are
bit-identical to the host twin below 2^40 (tests/test_gpu.py), so this is
the device's accuracy.

    python scripts/trig_accuracy_host.py [N per range]
"""
import json
import math
import os
import sys
from multiprocessing import Pool

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _cr(args):
    import mpmath
    mpmath.mp.prec = 200
    fn, xs = args
    f = mpmath.sin if fn == 0 else mpmath.cos
    return [float(f(mpmath.mpf(float(v)))) for v in xs]


def main():
    from deap_amd import _lib
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    rng = np.random.default_rng(0)
    near = (np.pi / 256) * rng.integers(1, 83000, n) + rng.uniform(-1e-9, 1e-9, n)
    ranges = {"u(-1,1)": rng.uniform(-1, 1, n),
              "u(-50,50)": rng.uniform(-50, 50, n),
              "u(-1024,1024)": rng.uniform(-1024, 1024, n),
              "near k*pi/256": near,
              "2^10..2^20": rng.uniform(1024, 2 ** 20, n) * rng.choice([-1, 1], n),
              "near k*pi/256, k < 2^26": (np.pi / 256) * rng.integers(83000, 2 ** 26, n)
              + rng.uniform(-1e-6, 1e-6, n),
              "2^20..2^30": rng.uniform(2 ** 20, 2 ** 30, n) * rng.choice([-1, 1], n),
              "2^30..2^40": rng.uniform(2 ** 30, 2 ** 40, n) * rng.choice([-1, 1], n)}
    out = {}
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        for name, x in ranges.items():
            for fn, fname in ((0, "sin"), (1, "cos")):
                chunks = np.array_split(x, 64)
                cr = np.concatenate([np.array(c) for c in
                                     pool.map(_cr, [(fn, c) for c in chunks])])
                dev = _lib.host_math(fn, x)
                lib = np.array([(math.sin if fn == 0 else math.cos)(v) for v in x])
                out["%s %s" % (fname, name)] = {
                    "n": len(x), "table_not_cr": int((dev != cr).sum()),
                    "glibc_not_cr": int((lib != cr).sum()),
                    "table_ne_glibc": int((dev != lib).sum())}
                print(fname, name, out["%s %s" % (fname, name)], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
