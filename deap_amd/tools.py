"""Population initialisers, selection and bookkeeping used around the GP path.

Behavioural restatement of the parts of the reference's ``deap/tools`` that the
GP examples wire around the evaluation hot path:

* initialisers ``initRepeat``/``initIterate``/``initCycle``
  (reference ``deap/tools/init.py:3-75``);
* selection ``selRandom``/``selBest``/``selWorst``/``selTournament``
  (reference ``deap/tools/selection.py:12-69``) and the lexicase family
  (``:214-320``, fed by per-case fitness from ``SymbRegCaseErrors``) —
  consumers of the fitness the GPU evaluator produces;
* ``Statistics``/``MultiStatistics``/``Logbook``/``HallOfFame``
  (reference ``deap/tools/support.py:154-589``).
"""
import random
from bisect import bisect_right
from collections import defaultdict
from copy import deepcopy
from functools import partial
from itertools import chain
from operator import attrgetter, eq

__all__ = ["initRepeat", "initIterate", "initCycle", "selRandom", "selBest",
           "selWorst", "selTournament", "selLexicase", "selEpsilonLexicase",
           "selAutomaticEpsilonLexicase", "selLexicaseGPU", "selEpsilonLexicaseGPU",
           "selAutomaticEpsilonLexicaseGPU", "selTournamentGPU", "Statistics",
           "MultiStatistics",
           "Logbook", "HallOfFame", "identity"]


# ----------------------------------------------------------------- init ----
def initRepeat(container, func, n):
    """``container(func() for _ in range(n))`` (reference init.py:3-25)."""
    return container(func() for _ in range(n))


def initIterate(container, generator):
    """``container(generator())`` (reference init.py:27-52)."""
    return container(generator())


def initCycle(container, seq_func, n=1):
    """Cycle through *seq_func* n times (reference init.py:54-75)."""
    return container(f() for _ in range(n) for f in seq_func)


# ------------------------------------------------------------ selection ----
def selRandom(individuals, k):
    return [random.choice(individuals) for _ in range(k)]


def selBest(individuals, k, fit_attr="fitness"):
    return sorted(individuals, key=attrgetter(fit_attr), reverse=True)[:k]


def selWorst(individuals, k, fit_attr="fitness"):
    return sorted(individuals, key=attrgetter(fit_attr))[:k]


def selTournament(individuals, k, tournsize, fit_attr="fitness"):
    """k tournaments of *tournsize* uniformly drawn aspirants; the first best
    aspirant wins each (reference selection.py:51-69)."""
    key = attrgetter(fit_attr)
    return [max(selRandom(individuals, tournsize), key=key)
            for _ in range(k)]


def _lexicase(individuals, k, survive):
    """Shared loop of the lexicase family (reference selection.py:214-320):
    per selection, shuffle the case indices, keep the candidates that
    ``survive(values, case, weight)`` case by case until one candidate or no
    case is left, then draw one candidate.  Same RNG calls, same order."""
    chosen = []
    for _ in range(k):
        weights = individuals[0].fitness.weights
        candidates = individuals
        cases = list(range(len(individuals[0].fitness.values)))
        random.shuffle(cases)
        while cases and len(candidates) > 1:
            c = cases[0]
            vals = [x.fitness.values[c] for x in candidates]
            keep = survive(vals, weights[c] > 0)
            candidates = [x for x, v in zip(candidates, vals) if keep(v)]
            cases.pop(0)
        chosen.append(random.choice(candidates))
    return chosen


def selLexicase(individuals, k):
    """Lexicase selection (reference selection.py:214-244): survivors of
    each case equal its best value."""
    def survive(vals, maximise):
        best = max(vals) if maximise else min(vals)
        return lambda v: v == best
    return _lexicase(individuals, k, survive)


def selEpsilonLexicase(individuals, k, epsilon):
    """epsilon-lexicase (reference selection.py:247-281): survivors are
    within *epsilon* of the best value of the case."""
    def survive(vals, maximise):
        if maximise:
            lim = max(vals) - epsilon
            return lambda v: v >= lim
        lim = min(vals) + epsilon
        return lambda v: v <= lim
    return _lexicase(individuals, k, survive)


def selAutomaticEpsilonLexicase(individuals, k):
    """Automatic epsilon-lexicase (reference selection.py:283-316): epsilon
    is the median absolute deviation of the case's values."""
    import numpy as np

    def survive(vals, maximise):
        med = np.median(vals)
        mad = np.median([abs(v - med) for v in vals])
        if maximise:
            lim = max(vals) - mad
            return lambda v: v >= lim
        lim = min(vals) + mad
        return lambda v: v <= lim
    return _lexicase(individuals, k, survive)


_LEX_CTX = {}


def _lexicase_gpu(individuals, k, mode, epsilon=0.0, device=None):
    """gpe_lexicase: the reference's selection loop on the GPU, drawing from
    the module ``random`` stream exactly as the reference does (its MT19937
    state goes to the device and comes back advanced), so a seeded run
    selects the same individuals and continues with the same stream."""
    import numpy as np
    from . import _lib
    from .evaluator import _default_device
    if k == 0:                            # the reference's loop runs 0 times
        return []
    if not individuals:                   # individuals[0] in the reference
        raise IndexError("list index out of range")
    dev = _default_device() if device is None else device
    if dev not in _LEX_CTX:
        _LEX_CTX[dev] = _lib.Context(dev)
    values = np.asarray([ind.fitness.values for ind in individuals],
                        dtype=np.float64)
    maximise = np.asarray(individuals[0].fitness.weights) > 0
    idx, failed = _LEX_CTX[dev].lexicase(values, maximise, k, random._inst,
                                         mode, epsilon)
    if failed >= 0:                       # random.choice([]) in the reference
        raise IndexError("Cannot choose from an empty sequence")
    return [individuals[i] for i in idx.tolist()]


def selLexicaseGPU(individuals, k, device=None):
    """Drop-in for :func:`selLexicase` (reference selection.py:214-244) that
    filters on the GPU; same selections, same ``random`` consumption."""
    return _lexicase_gpu(individuals, k, 0, device=device)


def selEpsilonLexicaseGPU(individuals, k, epsilon, device=None):
    """Drop-in for :func:`selEpsilonLexicase` (selection.py:247-281)."""
    return _lexicase_gpu(individuals, k, 1, epsilon, device=device)


# the device kernel keeps a case's values for the medians in LDS
AUTO_EPSILON_DEVICE_MAX = 16384


def selAutomaticEpsilonLexicaseGPU(individuals, k, device=None):
    """Drop-in for :func:`selAutomaticEpsilonLexicase`
    (selection.py:283-320).  Above AUTO_EPSILON_DEVICE_MAX individuals the
    selection runs as :func:`selAutomaticEpsilonLexicase` on the host (same
    selections, same ``random`` consumption; selection is not on the
    evaluation path)."""
    if len(individuals) > AUTO_EPSILON_DEVICE_MAX:
        return selAutomaticEpsilonLexicase(individuals, k)
    return _lexicase_gpu(individuals, k, 2, device=device)


# round 1's name of selLexicaseGPU, kept for callers written against it
selLexicaseDevice = selLexicaseGPU


def selTournamentGPU(individuals, k, tournsize, fit_attr="fitness",
                     device=None):
    """Drop-in for :func:`selTournament` (reference selection.py:51-69):
    the aspirants' ``random.choice`` draws are replayed on the GPU from the
    module ``random`` state (which comes back advanced), the winners picked
    there by ``Fitness`` order (wvalues); same selections, same stream."""
    import numpy as np
    from . import _lib
    from .evaluator import _default_device
    dev = _default_device() if device is None else device
    if dev not in _LEX_CTX:
        _LEX_CTX[dev] = _lib.Context(dev)
    if not individuals:                   # random.choice([]) in the reference
        if k > 0:
            raise IndexError("Cannot choose from an empty sequence")
        return []
    wv = np.asarray([getattr(ind, fit_attr).wvalues for ind in individuals],
                    dtype=np.float64)
    idx = _LEX_CTX[dev].tournament(wv, k, tournsize, random._inst)
    return [individuals[i] for i in idx.tolist()]


# -------------------------------------------------------------- support ----
def identity(obj):
    return obj


class Statistics(object):
    """Apply registered reductions to ``key(item)`` over a population
    (reference support.py:154-210)."""

    def __init__(self, key=identity):
        self.key = key
        self.functions = dict()
        self.fields = []

    def register(self, name, function, *args, **kargs):
        self.functions[name] = partial(function, *args, **kargs)
        self.fields.append(name)

    def compile(self, data):
        values = tuple(self.key(elem) for elem in data)
        return {name: fn(values) for name, fn in self.functions.items()}


class MultiStatistics(dict):
    """Named group of :class:`Statistics` (reference support.py:212-259)."""

    def compile(self, data):
        return {name: stats.compile(data) for name, stats in self.items()}

    @property
    def fields(self):
        return sorted(self.keys())

    def register(self, name, function, *args, **kargs):
        for stats in self.values():
            stats.register(name, function, *args, **kargs)


class Logbook(list):
    """Chronological list of record dicts; dict-valued entries become chapters
    (reference support.py:261-488)."""

    def __init__(self):
        self.buffindex = 0
        self.chapters = defaultdict(Logbook)
        self.columns_len = None
        self.header = None
        self.log_header = True

    def record(self, **infos):
        scalars = {k: v for k, v in infos.items() if not isinstance(v, dict)}
        for key, value in list(infos.items()):
            if isinstance(value, dict):
                sub = dict(value)
                sub.update(scalars)
                self.chapters[key].record(**sub)
                del infos[key]
        self.append(infos)

    def select(self, *names):
        if len(names) == 1:
            return [entry.get(names[0], None) for entry in self]
        return tuple([entry.get(n, None) for entry in self] for n in names)

    @property
    def stream(self):
        start, self.buffindex = self.buffindex, len(self)
        return self.__str__(start)

    def __delitem__(self, key):
        if isinstance(key, slice):
            for i in range(*key.indices(len(self))):
                self.pop(i)
                for chapter in self.chapters.values():
                    chapter.pop(i)
        else:
            self.pop(key)
            for chapter in self.chapters.values():
                chapter.pop(key)

    def pop(self, index=0):
        if index < self.buffindex:
            self.buffindex -= 1
        return super(Logbook, self).pop(index)

    def _lines(self, start):
        columns = self.header or (sorted(self[0].keys())
                                  + sorted(self.chapters.keys()))
        if not self.columns_len or len(self.columns_len) != len(columns):
            self.columns_len = [len(c) for c in columns]
        chapter_lines = {}
        offsets = defaultdict(int)
        for name, chapter in self.chapters.items():
            chapter_lines[name] = chapter._lines(start)
            if start == 0:
                offsets[name] = len(chapter_lines[name]) - len(self)
        rows = []
        for i, entry in enumerate(self[start:]):
            row = []
            for j, name in enumerate(columns):
                if name in chapter_lines:
                    cell = chapter_lines[name][i + offsets[name]]
                else:
                    value = entry.get(name, "")
                    cell = ("{0:n}" if isinstance(value, float)
                            else "{0}").format(value)
                self.columns_len[j] = max(self.columns_len[j], len(cell))
                row.append(cell)
            rows.append(row)
        if start == 0 and self.log_header:
            n_head = 1
            if len(self.chapters) > 0:
                n_head += max(len(v) for v in chapter_lines.values()) \
                    - len(self) + 1
            head = [[] for _ in range(n_head)]
            for j, name in enumerate(columns):
                if name in chapter_lines:
                    width = max(len(line.expandtabs())
                                for line in chapter_lines[name])
                    blanks = n_head - 2 - offsets[name]
                    for i in range(blanks):
                        head[i].append(" " * width)
                    head[blanks].append(name.center(width))
                    head[blanks + 1].append("-" * width)
                    for i in range(offsets[name]):
                        head[blanks + 2 + i].append(chapter_lines[name][i])
                else:
                    width = max([len(r[j].expandtabs()) for r in rows]
                                or [len(name)])
                    for line in head[:-1]:
                        line.append(" " * width)
                    head[-1].append(name)
            rows = list(chain(head, rows))
        template = "\t".join("{%d:<%d}" % (i, w)
                             for i, w in enumerate(self.columns_len))
        return [template.format(*row) for row in rows]

    def __str__(self, startindex=0):
        return "\n".join(self._lines(startindex))


class HallOfFame(object):
    """Best-ever individuals, kept sorted; ties keep the older entry first
    (reference support.py:490-589)."""

    def __init__(self, maxsize, similar=eq):
        self.maxsize = maxsize
        self.keys = list()
        self.items = list()
        self.similar = similar

    def update(self, population):
        for ind in population:
            if len(self) == 0 and self.maxsize != 0:
                self.insert(population[0])
                continue
            if ind.fitness > self[-1].fitness or len(self) < self.maxsize:
                if any(self.similar(ind, h) for h in self):
                    continue
                if len(self) >= self.maxsize:
                    self.remove(-1)
                self.insert(ind)

    def insert(self, item):
        item = deepcopy(item)
        i = bisect_right(self.keys, item.fitness)
        self.items.insert(len(self) - i, item)
        self.keys.insert(i, item.fitness)

    def remove(self, index):
        del self.keys[len(self) - (index % len(self) + 1)]
        del self.items[index]

    def clear(self):
        del self.items[:]
        del self.keys[:]

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]

    def __iter__(self):
        return iter(self.items)

    def __reversed__(self):
        return reversed(self.items)

    def __str__(self):
        return str(self.items)
