"""Lexicase selection: the DEAP-API host versions against the reference's
loops (same ``random`` stream), and the restatement of the device lexicase's
draws against the library's host twin (no GPU)."""
import random

import numpy as np
import pytest

from deap_amd import _lib, base, creator, tools
from oracle import selection_ref as ref


def population(values, weights):
    if not hasattr(creator, "FitLex%d" % len(weights)):
        creator.create("FitLex%d" % len(weights), base.Fitness,
                       weights=tuple(weights))
        creator.create("IndLex%d" % len(weights), list,
                       fitness=getattr(creator, "FitLex%d" % len(weights)))
    cls = getattr(creator, "IndLex%d" % len(weights))
    pop = []
    for i, row in enumerate(values):
        ind = cls([i])
        ind.fitness.values = tuple(row)
        pop.append(ind)
    return pop


def matrix(n, c, seed, levels=4):
    rng = np.random.default_rng(seed)
    return rng.integers(0, levels, size=(n, c)).astype(float).tolist()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sel_lexicase_matches_reference_loop(seed):
    values = matrix(60, 12, seed)
    weights = [-1.0] * 6 + [1.0] * 6
    pop = population(values, weights)
    random.seed(seed)
    got = [ind[0] for ind in tools.selLexicase(pop, 40)]
    random.seed(seed)
    assert got == ref.sel_lexicase_ref(values, weights, 40)


def test_sel_epsilon_lexicase_matches_reference_loop():
    values = (np.asarray(matrix(50, 9, 7, 50)) / 7.0).tolist()
    weights = [-1.0] * 9
    pop = population(values, weights)
    random.seed(11)
    got = [ind[0] for ind in tools.selEpsilonLexicase(pop, 30, 0.5)]
    random.seed(11)
    assert got == ref.sel_epsilon_lexicase_ref(values, weights, 30, 0.5)


def test_device_lexicase_draws_match_host_twin():
    rng = random.Random(5)
    for _ in range(300):
        seed, sel, draw = (rng.getrandbits(64), rng.getrandbits(20),
                           rng.getrandbits(32))
        m = rng.randrange(1, 2 ** 40)
        assert _lib.host_lex_draw(seed, sel, draw, m) == \
            ref.lex_below(ref.lex_draw(seed, sel, draw), m)
