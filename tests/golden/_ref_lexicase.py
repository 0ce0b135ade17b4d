#!/usr/bin/env python3
"""Golden selections of the REFERENCE's lexicase family.

Runs ``selLexicase``, ``selEpsilonLexicase`` and
``selAutomaticEpsilonLexicase`` (deap/tools/selection.py:214-320, the 2to3
copy made by ``make_oracle_copy.sh``) on committed fitness matrices under
fixed ``random.seed``s and records the selected indices plus a canary:
``random.getrandbits(32)`` drawn right after the call, which pins where the
reference left the random stream.  A case where the reference raises
(``random.choice([])`` after a nan) records the exception and the canary.

Build container only: ``python3 tests/golden/_ref_lexicase.py``
(writes ``lexicase.json.gz``).
"""
import gzip
import json
import os
import random
import sys
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_COPY = os.environ.get("DEAP_ORACLE_COPY", "/tmp/deap_oracle")
sys.path.insert(0, ORACLE_COPY)

from deap.tools import selection  # noqa: E402  (the reference)


def individuals(values, weights):
    return [SimpleNamespace(fitness=SimpleNamespace(values=tuple(row),
                                                    weights=tuple(weights)),
                            idx=i)
            for i, row in enumerate(values)]


def case(name, values, weights, k, seed, fn, **kw):
    pop = individuals(values, weights)
    random.seed(seed)
    err = None
    try:
        got = [ind.idx for ind in fn(pop, k, **kw)]
    except Exception as exc:          # IndexError: no candidate survived
        got, err = None, type(exc).__name__
    canary = random.getrandbits(32)
    return {"name": name, "values": [[float(v).hex() for v in row]
                                     for row in values],
            "weights": list(weights), "k": k, "seed": seed,
            "mode": {"selLexicase": 0, "selEpsilonLexicase": 1,
                     "selAutomaticEpsilonLexicase": 2}[fn.__name__],
            "epsilon": kw.get("epsilon", 0.0), "selected": got,
            "error": err, "canary": canary}


def main():
    rng = np.random.default_rng(2024)
    out = []
    v = rng.integers(0, 4, size=(60, 12)).astype(float)
    out.append(case("ties_mixed_weights", v, [-1.0] * 6 + [1.0] * 6, 40, 1,
                    selection.selLexicase))
    v = rng.integers(0, 3, size=(1000, 64)).astype(float)
    out.append(case("pop1000_cases64", v, [-1.0] * 64, 200, 2,
                    selection.selLexicase))
    v = rng.integers(0, 2, size=(50, 700)).astype(float)
    out.append(case("cases700_one_selection_past_624_words", v, [1.0] * 700,
                    5, 3, selection.selLexicase))
    v = rng.integers(0, 50, size=(50, 9)) / 7.0
    out.append(case("epsilon", v, [-1.0] * 9, 30, 4,
                    selection.selEpsilonLexicase, epsilon=0.5))
    v = rng.integers(0, 50, size=(50, 9)) / 7.0
    out.append(case("epsilon_maximise", v, [1.0] * 9, 30, 5,
                    selection.selEpsilonLexicase, epsilon=0.25))
    v = np.round(rng.normal(size=(40, 10)), 2)
    out.append(case("automatic_epsilon", v, [-1.0] * 10, 40, 6,
                    selection.selAutomaticEpsilonLexicase))
    v = np.round(rng.normal(size=(41, 7)), 1)
    out.append(case("automatic_epsilon_odd_maximise", v,
                    [1.0] * 3 + [-1.0] * 4, 25, 7,
                    selection.selAutomaticEpsilonLexicase))
    v = rng.integers(0, 3, size=(30, 5)).astype(float)
    v[0, :] = np.nan                  # a leading nan: no survivor
    out.append(case("leading_nan_raises", v, [-1.0] * 5, 10, 8,
                    selection.selLexicase))
    v = rng.integers(0, 3, size=(30, 5)).astype(float)
    v[7, 2] = np.nan                  # a later nan: never the best
    out.append(case("later_nan", v, [-1.0] * 5, 20, 9,
                    selection.selLexicase))
    path = os.path.join(HERE, "lexicase.json.gz")
    with gzip.open(path, "wt") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", path, [(c["name"], c["error"]) for c in out])


if __name__ == "__main__":
    main()
