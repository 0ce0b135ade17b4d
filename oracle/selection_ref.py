"""ORACLE — test infrastructure only, never the product path.

CPU restatements used as checkers for the selection side of the evaluator:

* ``sel_lexicase_ref`` / ``sel_epsilon_lexicase_ref``: the reference's loops
  (``deap/tools/selection.py:214-281``) written out directly on a matrix of
  fitness values — same ``random`` calls in the same order — to pin
  ``deap_amd.tools.selLexicase``/``selEpsilonLexicase``.
* ``device_lexicase_ref``: the device lexicase of ``gpeval.hip``
  (``lexicase_select``) restated with its counter-based draws
  (``lex_draw``/``lex_below``: splitmix64 finaliser, 128-bit product), so the
  GPU selection can be checked index for index.
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


def lex_draw(seed, sel, draw):
    """gpeval.hip lex_draw: splitmix64 finaliser of (seed, sel, draw)."""
    z = (seed ^ ((sel * 0xD1B54A32D192ED03) & M64)
         ^ ((draw * 0x9E3779B97F4A7C15) & M64)) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def lex_below(z, m):
    return (z * m) >> 64


def device_lexicase_ref(values, maximise, k, seed, epsilon=None):
    """The device algorithm: lazy Fisher-Yates case order, Python min/max
    semantics over candidates in index order, uniform final pick."""
    n, C = len(values), len(values[0])
    out = []
    for sel in range(k):
        cand = list(range(n))
        perm = list(range(C))
        t = 0
        while t < C and len(cand) > 1:
            r = t + lex_below(lex_draw(seed, sel, t), C - t)
            perm[t], perm[r] = perm[r], perm[t]
            c = perm[t]
            col = [values[i][c] for i in cand]
            finite = [v for v in col if not math.isnan(v)]
            if math.isnan(col[0]):
                best = col[0]
            elif maximise[c]:
                best = max(finite)
            else:
                best = min(finite)
            if epsilon is None:
                cand = [i for i, v in zip(cand, col) if v == best]
            elif maximise[c]:
                cand = [i for i, v in zip(cand, col) if v >= best - epsilon]
            else:
                cand = [i for i, v in zip(cand, col) if v <= best + epsilon]
            t += 1
        if not cand:
            out.append(-1)
            continue
        out.append(cand[lex_below(lex_draw(seed, sel, 0xFFFFFFFF),
                                  len(cand))])
    return out
