"""Device sin/cos/square vs glibc (Python math) vs correctly rounded (mpmath):
how often each is not correctly rounded, and how often device != glibc."""
import json
import math
import sys

import mpmath
import numpy as np

sys.path.insert(0, ".")
from deap_amd import _lib

mpmath.mp.prec = 200
rng = np.random.default_rng(0)
ctx = _lib.Context(0)
out = {}
for name, fn, gen in (("sin", 0, lambda n: rng.uniform(-50, 50, n)),
                      ("cos", 1, lambda n: rng.uniform(-50, 50, n)),
                      ("sin_small", 0, lambda n: rng.uniform(-1, 1, n)),
                      ("cos_small", 1, lambda n: rng.uniform(-1, 1, n)),
                      ("square", 2, lambda n: rng.uniform(-5, 5, n))):
    x = gen(20000)
    dev = ctx.math_probe(fn, x)
    if fn == 0:
        host = np.array([math.sin(v) for v in x])
        cr = np.array([float(mpmath.sin(mpmath.mpf(v))) for v in x])
    elif fn == 1:
        host = np.array([math.cos(v) for v in x])
        cr = np.array([float(mpmath.cos(mpmath.mpf(v))) for v in x])
    else:
        host = np.array([v ** 2 for v in x])
        cr = x * x
    out[name] = {"n": len(x), "dev_not_cr": int((dev != cr).sum()),
                 "glibc_not_cr": int((host != cr).sum()),
                 "dev_ne_glibc": int((dev != host).sum())}
print(json.dumps(out))
