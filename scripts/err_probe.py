import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
from deap_amd import _lib, configs, datasets
from deap_amd.flatten import Flattener
rng = np.random.default_rng(2024)
X = np.ascontiguousarray(rng.uniform(-1.0, 1.0, size=(2 ** 20, 10)).T)
y = datasets.unwrapped_ball_py(X)[None, :]
pset = configs.pset_for("symreg10")
pop = configs.population(pset, "half", 65536, 2024, 4, 8)
b = Flattener(pset).flatten(pop)
ctx = _lib.Context(0)
ctx.set_cases(_lib.GPE_MACHINE_F, X, y)
ctx.load_programs(b)
hi, lo, err, fl = ctx.run(_lib.GPE_MODE_MSE)
e = err[err != np.uint64(_lib.GPE_NO_ERROR)]
case = (e >> np.uint64(2)).astype(np.int64)
print("programs", len(err), "with a first error", len(e), "host err", int((b.err != 0).sum()))
if len(e):
    print("first-error case percentiles", np.percentile(case, [0, 10, 50, 90, 100]))
    L = np.asarray(b.length)[err != np.uint64(_lib.GPE_NO_ERROR)]
    print("their share of nodes %.4f" % (L.sum() / np.asarray(b.length).sum()))
    print("share of work after the first error (node-cases): %.4f" % ((L * (2**20 - case)).sum() / (np.asarray(b.length).sum() * 2**20)))
nonfin = ~np.isfinite(hi + lo)
print("non-finite sums", int(nonfin.sum()))
