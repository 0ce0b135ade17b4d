"""Runtime class factory (behaviour of the reference's ``deap/creator.py:96-171``).

``create("Individual", gp.PrimitiveTree, fitness=creator.FitnessMin)`` builds a
class in this module's namespace; attributes given as classes are instantiated
per instance, everything else becomes a class attribute.
"""
import warnings

__all__ = ["create"]


def create(name, base, **kargs):
    if name in globals():
        warnings.warn("A class named '{0}' has already been created and it "
                      "will be overwritten. Consider deleting previous "
                      "creation of that class or rename it.".format(name),
                      RuntimeWarning)

    per_instance = {k: v for k, v in kargs.items() if isinstance(v, type)}
    per_class = {k: v for k, v in kargs.items() if not isinstance(v, type)}

    def __init__(self, *args, **kw):
        for attr, cls in per_instance.items():
            setattr(self, attr, cls())
        if base.__init__ is not object.__init__:
            base.__init__(self, *args, **kw)

    new_type = type(str(name), (base,), per_class)
    new_type.__init__ = __init__
    new_type.__module__ = __name__
    globals()[name] = new_type
    return new_type
