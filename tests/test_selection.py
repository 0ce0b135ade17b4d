"""Lexicase selection: the DEAP-API host versions against the reference's
own selections (tests/golden/lexicase.json.gz, made by running the
reference's selection.py) and its loops, and the MT19937 replay the device
lexicase uses against CPython's ``random`` (no GPU)."""
import random

import numpy as np
import pytest

from deap_amd import _lib, base, creator, tools
from oracle import selection_ref as ref


def population(values, weights):
    tag = "%d_%x" % (len(weights), abs(hash(tuple(weights))))
    if not hasattr(creator, "FitLex" + tag):
        creator.create("FitLex" + tag, base.Fitness, weights=tuple(weights))
        creator.create("IndLex" + tag, list,
                       fitness=getattr(creator, "FitLex" + tag))
    cls = getattr(creator, "IndLex" + tag)
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


def test_mt_replay_is_cpython_random():
    """The draw arithmetic gpeval.hip's lexicase_mt replays (oracle
    MtReplay): shuffle and choice of CPython's random from its raw state."""
    rng = random.Random(123)
    for n_cases, k in ((12, 50), (700, 3), (1, 5), (64, 40)):
        mt = ref.MtReplay(rng.getstate()[1])
        for _ in range(k):
            cases = list(range(n_cases))
            rng.shuffle(cases)
            mine = list(range(n_cases))
            for i in reversed(range(1, n_cases)):
                j = mt.randbelow(i + 1)
                mine[i], mine[j] = mine[j], mine[i]
            assert mine == cases
            m = rng.randrange(1, 1000)
            assert 1 + mt.randbelow(999) == m
            assert mt.randbelow(m) == rng.choice(range(m))
        assert mt.state() == rng.getstate()[1]


@pytest.mark.parametrize("name", ["ties_mixed_weights", "pop1000_cases64",
                                  "cases700_one_selection_past_624_words",
                                  "epsilon", "epsilon_maximise",
                                  "automatic_epsilon",
                                  "automatic_epsilon_odd_maximise",
                                  "leading_nan_raises", "later_nan"])
def test_host_lexicase_matches_reference_fixtures(name):
    """deap_amd.tools' lexicase family against the reference's own
    selections (indices and the random stream position after them)."""
    from conftest import load_golden
    g = {c["name"]: c for c in load_golden("lexicase")}[name]
    values = [[float.fromhex(v) for v in row] for row in g["values"]]
    pop = population(values, g["weights"])
    fn = {0: tools.selLexicase, 1: tools.selEpsilonLexicase,
          2: tools.selAutomaticEpsilonLexicase}[g["mode"]]
    kw = {"epsilon": g["epsilon"]} if g["mode"] == 1 else {}
    random.seed(g["seed"])
    if g["error"]:
        with pytest.raises(IndexError):
            fn(pop, g["k"], **kw)
    else:
        assert [ind[0] for ind in fn(pop, g["k"], **kw)] == g["selected"]
    assert random.getrandbits(32) == g["canary"]


TOURN_CASES = ["symbreg_like_min", "hits_max_ties",
               "two_objectives_lexicographic", "n_4097_rejections",
               "pop_20000_past_624_words", "single_individual"]


@pytest.mark.parametrize("name", TOURN_CASES)
def test_tournament_oracle_and_host_match_reference_fixtures(name):
    """The oracle's selTournament restatement (MtReplay draws) and
    deap_amd.tools.selTournament against the reference's own selections
    (tests/golden/tournament.json.gz, made by _ref_tournament.py): indices
    and the random stream position after them."""
    from conftest import load_golden
    g = {c["name"]: c for c in load_golden("tournament")}[name]
    values = [[float.fromhex(v) for v in row] for row in g["values"]]
    wv = [[v * w for v, w in zip(row, g["weights"])] for row in values]
    random.seed(g["seed"])
    mt = ref.MtReplay(random.getstate()[1])
    assert ref.sel_tournament_ref(wv, g["k"], g["tournsize"], mt) == \
        g["selected"]
    r = random.Random()
    r.setstate((3, mt.state(), None))
    assert r.getrandbits(32) == g["canary"]
    pop = population(values, g["weights"])
    random.seed(g["seed"])
    got = tools.selTournament(pop, g["k"], g["tournsize"])
    assert [ind[0] for ind in got] == g["selected"]
    assert random.getrandbits(32) == g["canary"]
