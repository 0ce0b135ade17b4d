#!/usr/bin/env python3
"""Golden selections of the REFERENCE's ``selTournament``
(deap/tools/selection.py:51-69, ``selRandom`` :15-28: ``random.choice`` per
aspirant, ``max`` by fitness) on committed fitness matrices under fixed
``random.seed``s, plus a canary ``random.getrandbits(32)`` drawn right after
the call (where the reference left the random stream).  The individuals'
``fitness`` are the reference's own ``base.Fitness`` subclasses, so ``max``
compares them exactly as the reference does (``wvalues`` tuples).

Build container only: ``python3 tests/golden/_ref_tournament.py`` (needs the
2to3 copy from ``make_oracle_copy.sh``; writes ``tournament.json.gz``).
"""
import gzip
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_COPY = os.environ.get("DEAP_ORACLE_COPY", "/tmp/deap_oracle")
sys.path.insert(0, ORACLE_COPY)

from deap import base  # noqa: E402  (the reference)
from deap.tools import selection  # noqa: E402


class Ind(object):
    def __init__(self, idx, fitness):
        self.idx = idx
        self.fitness = fitness


def case(name, values, weights, k, tournsize, seed):
    fit_cls = type("Fit", (base.Fitness,), {"weights": tuple(weights)})
    pop = []
    for i, row in enumerate(values):
        f = fit_cls()
        f.values = tuple(float(v) for v in row)
        pop.append(Ind(i, f))
    random.seed(seed)
    got = [ind.idx for ind in selection.selTournament(pop, k, tournsize)]
    canary = random.getrandbits(32)
    return {"name": name, "values": [[float(v).hex() for v in row]
                                     for row in values],
            "weights": list(weights), "k": k, "tournsize": tournsize,
            "seed": seed, "selected": got, "canary": canary}


def main():
    rng = np.random.default_rng(77)
    out = []
    v = rng.integers(0, 50, size=(300, 1)) / 7.0
    out.append(case("symbreg_like_min", v, [-1.0], 300, 3, 318))
    v = rng.integers(0, 64, size=(1000, 1)).astype(float)
    out.append(case("hits_max_ties", v, [1.0], 1000, 7, 21))
    v = rng.integers(0, 5, size=(257, 2)).astype(float)
    out.append(case("two_objectives_lexicographic", v, [1.0, -1.0], 100, 4, 5))
    v = rng.normal(size=(4097, 1))
    out.append(case("n_4097_rejections", v, [-1.0], 5000, 2, 99))
    v = rng.integers(0, 3, size=(20000, 1)).astype(float)
    out.append(case("pop_20000_past_624_words", v, [1.0], 40000, 3, 2024))
    v = rng.normal(size=(1, 1))
    out.append(case("single_individual", v, [1.0], 5, 3, 1))
    path = os.path.join(HERE, "tournament.json.gz")
    with gzip.open(path, "wt") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", path, [c["name"] for c in out])


if __name__ == "__main__":
    main()
