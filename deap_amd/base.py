"""Toolbox and Fitness — the drop-in boundary of the GP evaluation path.

Clean-room restatement of the behaviour of the reference's ``deap/base.py``:

* ``Toolbox`` (reference ``deap/base.py:48-122``) is an alias registry that wraps
  callables in ``functools.partial``.  Its default ``map`` is the builtin ``map``
  (``base.py:50``); the GPU evaluator plugs in by registering ``map`` and
  ``evaluate`` (see :mod:`deap_amd.evaluator`).
* ``Fitness`` (reference ``deap/base.py:125-270``) stores weighted values and
  compares them lexicographically.  The GPU evaluator hands back 1-tuples that
  are assigned through the ``values`` setter (``base.py:187-198``).
"""
import copy
from collections.abc import Sequence
from functools import partial
from operator import mul, truediv

__all__ = ["Toolbox", "Fitness"]


class Toolbox(object):
    """Registry of evolutionary operators (reference ``base.py:34-122``)."""

    def __init__(self):
        self.register("clone", copy.deepcopy)
        self.register("map", map)

    def register(self, alias, function, *args, **kargs):
        """Bind ``partial(function, *args, **kargs)`` under *alias*."""
        bound = partial(function, *args, **kargs)
        bound.__name__ = alias
        bound.__doc__ = function.__doc__
        # Classes keep their own dict; plain callables share theirs
        # (reference base.py:84-88).
        if hasattr(function, "__dict__") and not isinstance(function, type):
            bound.__dict__.update(dict(function.__dict__))
        setattr(self, alias, bound)

    def unregister(self, alias):
        delattr(self, alias)

    def decorate(self, alias, *decorators):
        """Re-register *alias* with its function wrapped by *decorators*,
        keeping the bound arguments (reference ``base.py:100-122``)."""
        bound = getattr(self, alias)
        func = bound.func
        for deco in decorators:
            func = deco(func)
        self.register(alias, func, *bound.args, **bound.keywords)


class Fitness(object):
    """Weighted, lexicographically compared fitness (reference ``base.py:125``).

    Subclasses (made by :func:`deap_amd.creator.create`) set ``weights``.
    """

    weights = None
    wvalues = ()

    def __init__(self, values=()):
        if self.weights is None:
            raise TypeError("Can't instantiate abstract %r with abstract "
                            "attribute weights." % (self.__class__))
        if not isinstance(self.weights, Sequence):
            raise TypeError("Attribute weights of %r must be a sequence."
                            % self.__class__)
        if len(values) > 0:
            self.values = values

    def getValues(self):
        return tuple(map(truediv, self.wvalues, self.weights))

    def setValues(self, values):
        assert len(values) == len(self.weights), \
            "Assigned values have not the same length than fitness weights"
        try:
            self.wvalues = tuple(map(mul, values, self.weights))
        except TypeError as exc:
            raise TypeError("Both weights and assigned values must be a "
                            "sequence of numbers when assigning to values of "
                            "%r. Currently assigning value(s) %r of %r to a "
                            "fitness with weights %s."
                            % (self.__class__, values, type(values),
                               self.weights)) from exc

    def delValues(self):
        self.wvalues = ()

    values = property(getValues, setValues, delValues)

    def dominates(self, other, obj=slice(None)):
        strictly_better = False
        for mine, theirs in zip(self.wvalues[obj], other.wvalues[obj]):
            if mine > theirs:
                strictly_better = True
            elif mine < theirs:
                return False
        return strictly_better

    @property
    def valid(self):
        return len(self.wvalues) != 0

    def __hash__(self):
        return hash(self.wvalues)

    def __gt__(self, other):
        return not self.__le__(other)

    def __ge__(self, other):
        return not self.__lt__(other)

    def __le__(self, other):
        return self.wvalues <= other.wvalues

    def __lt__(self, other):
        return self.wvalues < other.wvalues

    def __eq__(self, other):
        return self.wvalues == other.wvalues

    def __ne__(self, other):
        return not self.__eq__(other)

    def __deepcopy__(self, memo):
        twin = self.__class__()
        twin.wvalues = self.wvalues
        return twin

    def __str__(self):
        return str(self.values if self.valid else tuple())

    def __repr__(self):
        return "%s.%s(%r)" % (self.__module__, self.__class__.__name__,
                              self.values if self.valid else tuple())
