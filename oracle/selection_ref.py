"""ORACLE — test infrastructure only, never the product path.

CPU restatements used as checkers for the selection side of the evaluator:

* ``sel_lexicase_ref`` / ``sel_epsilon_lexicase_ref``: the reference's loops
  (``deap/tools/selection.py:214-281``) written out directly on a matrix of
  fitness values — same ``random`` calls in the same order — to pin
  ``deap_amd.tools.selLexicase``/``selEpsilonLexicase``.
* ``MtReplay``: CPython's MT19937 (``Modules/_randommodule.c``
  genrand_uint32, ``random.py`` _randbelow_with_getrandbits) driven from the
  raw state words of ``random.getstate()`` — the draw arithmetic the device
  lexicase (``gpeval.hip`` lexicase_mt) replays; pinned against the
  ``random`` module itself by tests/test_selection.py.
* ``sel_tournament_ref``: ``selTournament`` (``selection.py:51-69``, with
  ``selRandom`` :15-28) on a matrix of weighted fitness values, drawing
  from an ``MtReplay`` — the device tournament's restatement, pinned by the
  reference-generated ``tests/golden/tournament.json.gz``.
"""
import math
import random

M64 = (1 << 64) - 1


def sel_lexicase_ref(values, weights, k):
    """values[i][c]; returns selected row indices (reference :214-244)."""
    out = []
    for _ in range(k):
        candidates = list(range(len(values)))
        cases = list(range(len(values[0])))
        random.shuffle(cases)
        while len(cases) > 0 and len(candidates) > 1:
            f = max if weights[cases[0]] > 0 else min
            best = f(map(lambda i: values[i][cases[0]], candidates))
            candidates = list(filter(lambda i: values[i][cases[0]] == best,
                                     candidates))
            cases.pop(0)
        out.append(random.choice(candidates))
    return out


def sel_epsilon_lexicase_ref(values, weights, k, epsilon):
    """Reference :247-281 on a value matrix."""
    out = []
    for _ in range(k):
        candidates = list(range(len(values)))
        cases = list(range(len(values[0])))
        random.shuffle(cases)
        while len(cases) > 0 and len(candidates) > 1:
            col = [values[i][cases[0]] for i in candidates]
            if weights[cases[0]] > 0:
                lim = max(col) - epsilon
                candidates = [i for i in candidates
                              if values[i][cases[0]] >= lim]
            else:
                lim = min(col) + epsilon
                candidates = [i for i in candidates
                              if values[i][cases[0]] <= lim]
            cases.pop(0)
        out.append(random.choice(candidates))
    return out


class MtReplay(object):
    """genrand_uint32 / getrandbits(k <= 32) / _randbelow on raw MT19937
    state words (random.getstate()[1]: 624 words + position)."""
    N, M = 624, 397

    def __init__(self, words):
        self.mt = [int(w) & 0xFFFFFFFF for w in words[:self.N]]
        self.idx = int(words[self.N])

    def _twist(self):
        mt, N, M = self.mt, self.N, self.M
        for kk in range(N):
            y = (mt[kk] & 0x80000000) | (mt[(kk + 1) % N] & 0x7FFFFFFF)
            mt[kk] = mt[(kk + M) % N] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.idx = 0

    def genrand(self):
        if self.idx >= self.N:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        return (y ^ (y >> 18)) & 0xFFFFFFFF

    def randbelow(self, n):
        if not n:
            return 0
        k = n.bit_length()
        r = self.genrand() >> (32 - k)
        while r >= n:
            r = self.genrand() >> (32 - k)
        return r

    def state(self):
        return tuple(self.mt) + (self.idx,)


def wvalues_gt(a, b):
    """``Fitness.__gt__`` (deap/base.py:218-219): not (a.wvalues <=
    b.wvalues), Python tuple order (distinct float objects)."""
    for x, y in zip(a, b):
        if x == y:
            continue
        return not (x <= y)
    return not (len(a) <= len(b))


def sel_tournament_ref(wvalues, k, tournsize, mt):
    """Reference :51-69: k tournaments of ``tournsize`` aspirants drawn with
    ``random.choice`` (``mt.randbelow(n)`` each), ``max`` keeping the first
    of equal fitnesses.  Returns the selected row indices; ``mt`` advances."""
    n = len(wvalues)
    out = []
    for _ in range(k):
        asp = [mt.randbelow(n) for _ in range(tournsize)]
        best = asp[0]
        for c in asp[1:]:
            if wvalues_gt(wvalues[c], wvalues[best]):
                best = c
        out.append(best)
    return out
