"""Genetic-programming representation, generation and variation.

A restatement of the parts of the reference's ``deap/gp.py`` that the GP
evaluation path and its callers consume.  It follows the reference statement
for statement where the random-number consumption or the error messages must
match (``generate``, ``cxOnePoint``, ``PrimitiveTree`` parsing): the prefix
``PrimitiveTree`` (``gp.py:44-184``),
its node classes (``gp.py:187-257``), primitive sets (``gp.py:260-456``),
``compile`` (``gp.py:462-487``), tree generation (``gp.py:519-638``) and the
variation operators used by ``eaSimple``/``varAnd`` (``gp.py:645-931``).

Random-number consumption mirrors the reference call for call (same
``random.choice``/``randint``/``random`` calls on sequences of the same length),
so that seeded runs reproduce the reference's populations exactly — the
config-1 logbook test relies on it.

``compile`` is kept for API completeness (it is the per-individual path the
GPU evaluator replaces); the evaluator itself never calls it.
"""
import copy
import random
import re
import sys
from collections import defaultdict, deque
from functools import wraps
from inspect import isclass

__type__ = object

__all__ = ["PrimitiveTree", "Primitive", "Terminal", "Ephemeral",
           "PrimitiveSetTyped", "PrimitiveSet", "compile", "compileADF",
           "genFull", "genGrow", "genHalfAndHalf", "genRamped", "generate",
           "cxOnePoint", "cxOnePointLeafBiased", "mutUniform",
           "mutNodeReplacement", "mutEphemeral", "mutInsert", "mutShrink",
           "staticLimit"]


# --------------------------------------------------------------------------
# Tree and node types
# --------------------------------------------------------------------------
class PrimitiveTree(list):
    """A GP tree stored as a list of nodes in prefix (root-first) order
    (reference ``gp.py:44-184``)."""

    def __init__(self, content):
        list.__init__(self, content)

    def __deepcopy__(self, memo):
        # Nodes are immutable and shared; only the instance dict (fitness)
        # is deep-copied (reference gp.py:58-61).
        twin = self.__class__(self)
        twin.__dict__.update(copy.deepcopy(self.__dict__, memo))
        return twin

    def __setitem__(self, key, val):
        if isinstance(key, slice):
            if key.start >= len(self):
                raise IndexError("Invalid slice object (try to assign a %s"
                                 " in a tree of size %d)." % (key, len(self)))
            open_slots = val[0].arity
            for node in val[1:]:
                open_slots += node.arity - 1
            if open_slots != 0:
                raise ValueError("Invalid slice assignation : insertion of"
                                 " an incomplete subtree is not allowed in "
                                 "PrimitiveTree.")
        elif val.arity != self[key].arity:
            raise ValueError("Invalid node replacement with a node of a"
                             " different arity.")
        list.__setitem__(self, key, val)

    def __str__(self):
        """Python-expression rendering, e.g. ``add(x, mul(x, 1))``."""
        pending = []          # [node, rendered-args]
        text = ""
        for node in self:
            pending.append([node, []])
            while len(pending[-1][1]) == pending[-1][0].arity:
                node_, args = pending.pop()
                text = node_.format(*args)
                if not pending:
                    break
                pending[-1][1].append(text)
        return text

    @classmethod
    def from_string(cls, string, pset):
        """Parse the output of ``str(tree)`` back into a tree
        (reference ``gp.py:106-153``)."""
        tokens = re.split("[ \t\n\r\f\v(),]", string)
        nodes = []
        expected = deque()
        for token in tokens:
            if token == "":
                continue
            type_ = expected.popleft() if expected else None
            if token in pset.mapping:
                prim = pset.mapping[token]
                if type_ is not None and not issubclass(prim.ret, type_):
                    raise TypeError("Primitive {} return type {} does not "
                                    "match the expected one: {}."
                                    .format(prim, prim.ret, type_))
                nodes.append(prim)
                if isinstance(prim, Primitive):
                    expected.extendleft(reversed(prim.args))
            else:
                try:
                    value = eval(token)
                except NameError:
                    raise TypeError("Unable to evaluate terminal: {}."
                                    .format(token))
                if type_ is None:
                    type_ = type(value)
                if not issubclass(type(value), type_):
                    raise TypeError("Terminal {} type {} does not "
                                    "match the expected one: {}."
                                    .format(value, type(value), type_))
                nodes.append(Terminal(value, False, type_))
        return cls(nodes)

    @property
    def height(self):
        """Depth of the deepest node (root has depth 0)."""
        depths = [0]
        deepest = 0
        for node in self:
            d = depths.pop()
            if d > deepest:
                deepest = d
            depths.extend([d + 1] * node.arity)
        return deepest

    @property
    def root(self):
        return self[0]

    def searchSubtree(self, begin):
        """Slice covering the subtree rooted at index *begin*."""
        end = begin + 1
        need = self[begin].arity
        while need > 0:
            need += self[end].arity - 1
            end += 1
        return slice(begin, end)


class Primitive(object):
    """Function node (reference ``gp.py:187-213``).

        >>> Primitive("mul", (int, int), int).format(1, 2)
        'mul(1, 2)'
    """
    __slots__ = ("name", "arity", "args", "ret", "seq")

    def __init__(self, name, args, ret):
        self.name = name
        self.arity = len(args)
        self.args = args
        self.ret = ret
        placeholders = ", ".join("{%d}" % i for i in range(self.arity))
        self.seq = "%s(%s)" % (self.name, placeholders)

    def format(self, *args):
        return self.seq.format(*args)

    def __eq__(self, other):
        if type(self) is type(other):
            return all(getattr(self, s) == getattr(other, s)
                       for s in self.__slots__)
        return NotImplemented

    __hash__ = object.__hash__


class Terminal(object):
    """Leaf node: an argument, a named/literal constant (``gp.py:216-240``)."""
    __slots__ = ("name", "value", "ret", "conv_fct")

    def __init__(self, terminal, symbolic, ret):
        self.ret = ret
        self.value = terminal
        self.name = str(terminal)
        self.conv_fct = str if symbolic else repr

    @property
    def arity(self):
        return 0

    def format(self):
        return self.conv_fct(self.value)

    def __eq__(self, other):
        if type(self) is type(other):
            return all(getattr(self, s) == getattr(other, s)
                       for s in self.__slots__)
        return NotImplemented

    __hash__ = object.__hash__


class Ephemeral(Terminal):
    """Terminal whose value is drawn once when the node is created
    (``gp.py:243-257``).  Concrete subclasses are made by
    ``addEphemeralConstant`` and live in this module's namespace so that
    trees pickle (reference ``gp.py:393-397``)."""

    def __init__(self):
        Terminal.__init__(self, self.func(), symbolic=False, ret=self.ret)

    @staticmethod
    def func():
        raise NotImplementedError


# --------------------------------------------------------------------------
# Primitive sets
# --------------------------------------------------------------------------
class PrimitiveSetTyped(object):
    """Strongly-typed primitive set (reference ``gp.py:260-429``).

    ``primitives``/``terminals`` map a type to the list of nodes returning a
    subclass of it; list order matters because generation draws from it with
    ``random.choice``.
    """

    def __init__(self, name, in_types, ret_type, prefix="ARG"):
        self.terminals = defaultdict(list)
        self.primitives = defaultdict(list)
        self.arguments = []
        self.context = {"__builtins__": None}
        self.mapping = dict()
        self.terms_count = 0
        self.prims_count = 0
        self.name = name
        self.ret = ret_type
        self.ins = in_types
        for i, type_ in enumerate(in_types):
            arg = "%s%d" % (prefix, i)
            self.arguments.append(arg)
            self._add(Terminal(arg, True, type_))
            self.terms_count += 1

    def renameArguments(self, **kargs):
        for i, old in enumerate(self.arguments):
            if old in kargs:
                new = kargs[old]
                self.arguments[i] = new
                self.mapping[new] = self.mapping.pop(old)
                self.mapping[new].value = new

    @staticmethod
    def _ensure_type(table, type_):
        # A new type inherits every node already registered under one of its
        # subclasses, in registration order.
        if type_ in table:
            return
        merged = []
        for known, nodes in table.items():
            if issubclass(known, type_):
                for node in nodes:
                    if node not in merged:
                        merged.append(node)
        table[type_] = merged

    def _add(self, node):
        self._ensure_type(self.primitives, node.ret)
        self._ensure_type(self.terminals, node.ret)
        if isinstance(node, Primitive):
            self.mapping[node.name] = node
            for t in node.args:
                self._ensure_type(self.primitives, t)
                self._ensure_type(self.terminals, t)
            table = self.primitives
        else:
            if not isclass(node):          # ephemeral classes have no name
                self.mapping[node.name] = node
            table = self.terminals
        for type_ in table:
            if issubclass(node.ret, type_):
                table[type_].append(node)

    def addPrimitive(self, primitive, in_types, ret_type, name=None):
        if name is None:
            name = primitive.__name__
        prim = Primitive(name, in_types, ret_type)
        assert name not in self.context or self.context[name] is primitive, \
            "Primitives are required to have a unique name. Consider using " \
            "the argument 'name' to rename your second '%s' primitive." % name
        self._add(prim)
        self.context[prim.name] = primitive
        self.prims_count += 1

    def addTerminal(self, terminal, ret_type, name=None):
        symbolic = False
        if name is None and callable(terminal):
            name = terminal.__name__
        assert name not in self.context, \
            "Terminals are required to have a unique name. Consider using " \
            "the argument 'name' to rename your second %s terminal." % name
        if name is not None:
            self.context[name] = terminal
            terminal = name
            symbolic = True
        elif terminal in (True, False):
            self.context[str(terminal)] = terminal
        self._add(Terminal(terminal, symbolic, ret_type))
        self.terms_count += 1

    def addEphemeralConstant(self, name, ephemeral, ret_type):
        registry = globals()
        if name not in registry:
            cls = type(name, (Ephemeral,), {"func": staticmethod(ephemeral),
                                            "ret": ret_type})
            registry[name] = cls
        else:
            cls = registry[name]
            if isclass(cls) and issubclass(cls, Ephemeral):
                if cls.func is not ephemeral:
                    raise Exception("Ephemerals with different functions "
                                    "should be named differently, even "
                                    "between psets.")
                if cls.ret is not ret_type:
                    raise Exception("Ephemerals with the same name and "
                                    "function should have the same type, "
                                    "even between psets.")
            else:
                raise Exception("Ephemerals should be named differently "
                                "than classes defined in the gp module.")
        self._add(cls)
        self.terms_count += 1

    def addADF(self, adfset):
        self._add(Primitive(adfset.name, adfset.ins, adfset.ret))
        self.prims_count += 1

    @property
    def terminalRatio(self):
        return self.terms_count / float(self.terms_count + self.prims_count)


class PrimitiveSet(PrimitiveSetTyped):
    """Loosely-typed primitive set (reference ``gp.py:432-456``)."""

    def __init__(self, name, arity, prefix="ARG"):
        PrimitiveSetTyped.__init__(self, name, [__type__] * arity, __type__,
                                   prefix)

    def addPrimitive(self, primitive, arity, name=None):
        assert arity > 0, "arity should be >= 1"
        PrimitiveSetTyped.addPrimitive(self, primitive, [__type__] * arity,
                                       __type__, name)

    def addTerminal(self, terminal, name=None):
        PrimitiveSetTyped.addTerminal(self, terminal, __type__, name)

    def addEphemeralConstant(self, name, ephemeral):
        PrimitiveSetTyped.addEphemeralConstant(self, name, ephemeral,
                                               __type__)


# --------------------------------------------------------------------------
# Compilation (the per-individual path the GPU evaluator replaces)
# --------------------------------------------------------------------------
def compile(expr, pset):
    """Tree → Python callable via ``eval`` (reference ``gp.py:462-487``)."""
    code = str(expr)
    if len(pset.arguments) > 0:
        code = "lambda %s: %s" % (",".join(pset.arguments), code)
    return eval(code, pset.context, {})


def compileADF(expr, psets):
    """Compile a main tree plus its ADFs (reference ``gp.py:490-513``)."""
    adfs = {}
    func = None
    for pset, subexpr in reversed(list(zip(psets, expr))):
        pset.context.update(adfs)
        func = compile(subexpr, pset)
        adfs[pset.name] = func
    return func


# --------------------------------------------------------------------------
# Generation
# --------------------------------------------------------------------------
def generate(pset, min_, max_, condition, type_=None):
    """Depth-first random tree construction (reference ``gp.py:589-638``)."""
    if type_ is None:
        type_ = pset.ret
    expr = []
    height = random.randint(min_, max_)
    todo = [(0, type_)]
    while todo:
        depth, want = todo.pop()
        if condition(height, depth):
            try:
                term = random.choice(pset.terminals[want])
            except IndexError as exc:
                raise IndexError("The gp.generate function tried to add a "
                                 "terminal of type '%s', but there is none "
                                 "available." % (want,)).with_traceback(
                                     sys.exc_info()[2]) from exc
            if isclass(term):
                term = term()
            expr.append(term)
        else:
            try:
                prim = random.choice(pset.primitives[want])
            except IndexError as exc:
                raise IndexError("The gp.generate function tried to add a "
                                 "primitive of type '%s', but there is none "
                                 "available." % (want,)).with_traceback(
                                     sys.exc_info()[2]) from exc
            expr.append(prim)
            for arg in reversed(prim.args):
                todo.append((depth + 1, arg))
    return expr


def genFull(pset, min_, max_, type_=None):
    """All leaves at the same depth (reference ``gp.py:519-536``)."""
    return generate(pset, min_, max_, lambda height, depth: depth == height,
                    type_)


def genGrow(pset, min_, max_, type_=None):
    """Leaves at varying depths (reference ``gp.py:539-559``)."""
    def stop(height, depth):
        return depth == height or \
            (depth >= min_ and random.random() < pset.terminalRatio)
    return generate(pset, min_, max_, stop, type_)


def genHalfAndHalf(pset, min_, max_, type_=None):
    """genGrow or genFull with equal probability (``gp.py:562-576``)."""
    method = random.choice((genGrow, genFull))
    return method(pset, min_, max_, type_)


def genRamped(pset, min_, max_, type_=None):
    return genHalfAndHalf(pset, min_, max_, type_)


# --------------------------------------------------------------------------
# Variation
# --------------------------------------------------------------------------
def cxOnePoint(ind1, ind2):
    """Swap two random same-typed subtrees (reference ``gp.py:645-682``)."""
    if len(ind1) < 2 or len(ind2) < 2:
        return ind1, ind2
    sites1 = defaultdict(list)
    sites2 = defaultdict(list)
    if ind1.root.ret == __type__:
        sites1[__type__] = range(1, len(ind1))
        sites2[__type__] = range(1, len(ind2))
        shared = [__type__]
    else:
        for i, node in enumerate(ind1[1:], 1):
            sites1[node.ret].append(i)
        for i, node in enumerate(ind2[1:], 1):
            sites2[node.ret].append(i)
        shared = set(sites1.keys()).intersection(set(sites2.keys()))
    if len(shared) > 0:
        type_ = random.choice(list(shared))
        i1 = random.choice(sites1[type_])
        i2 = random.choice(sites2[type_])
        s1 = ind1.searchSubtree(i1)
        s2 = ind2.searchSubtree(i2)
        ind1[s1], ind2[s2] = ind2[s2], ind1[s1]
    return ind1, ind2


def cxOnePointLeafBiased(ind1, ind2, termpb):
    """Koza-style leaf-biased one point crossover (``gp.py:685-737``)."""
    if len(ind1) < 2 or len(ind2) < 2:
        return ind1, ind2
    want_leaf1 = random.random() < termpb
    want_leaf2 = random.random() < termpb
    sites1 = defaultdict(list)
    sites2 = defaultdict(list)
    for i, node in enumerate(ind1[1:], 1):
        if (node.arity == 0) == want_leaf1:
            sites1[node.ret].append(i)
    for i, node in enumerate(ind2[1:], 1):
        if (node.arity == 0) == want_leaf2:
            sites2[node.ret].append(i)
    shared = set(sites1.keys()).intersection(set(sites2.keys()))
    if len(shared) > 0:
        type_ = random.sample(tuple(shared), 1)[0]
        i1 = random.choice(sites1[type_])
        i2 = random.choice(sites2[type_])
        s1 = ind1.searchSubtree(i1)
        s2 = ind2.searchSubtree(i2)
        ind1[s1], ind2[s2] = ind2[s2], ind1[s1]
    return ind1, ind2


def mutUniform(individual, expr, pset):
    """Replace a random subtree by a fresh one (reference ``gp.py:743-757``)."""
    index = random.randrange(len(individual))
    where = individual.searchSubtree(index)
    type_ = individual[index].ret
    individual[where] = expr(pset=pset, type_=type_)
    return individual,


def mutNodeReplacement(individual, pset):
    """Swap one node for another of the same arity (``gp.py:760-783``)."""
    if len(individual) < 2:
        return individual,
    index = random.randrange(1, len(individual))
    node = individual[index]
    if node.arity == 0:
        term = random.choice(pset.terminals[node.ret])
        if isclass(term):
            term = term()
        individual[index] = term
    else:
        same = [p for p in pset.primitives[node.ret] if p.args == node.args]
        individual[index] = random.choice(same)
    return individual,


def mutEphemeral(individual, mode):
    """Redraw one or all ephemeral constants (``gp.py:786-811``)."""
    if mode not in ["one", "all"]:
        raise ValueError("Mode must be one of \"one\" or \"all\"")
    where = [i for i, node in enumerate(individual)
             if isinstance(node, Ephemeral)]
    if len(where) > 0:
        if mode == "one":
            where = (random.choice(where),)
        for i in where:
            individual[i] = type(individual[i])()
    return individual,


def mutInsert(individual, pset):
    """Insert a new primitive above a random node (``gp.py:814-851``)."""
    index = random.randrange(len(individual))
    node = individual[index]
    where = individual.searchSubtree(index)
    candidates = [p for p in pset.primitives[node.ret] if node.ret in p.args]
    if len(candidates) == 0:
        return individual,
    new_node = random.choice(candidates)
    children = [None] * len(new_node.args)
    keep_at = random.choice([i for i, a in enumerate(new_node.args)
                             if a == node.ret])
    for i, arg_type in enumerate(new_node.args):
        if i != keep_at:
            term = random.choice(pset.terminals[arg_type])
            if isclass(term):
                term = term()
            children[i] = term
    children[keep_at:keep_at + 1] = individual[where]
    children.insert(0, new_node)
    individual[where] = children
    return individual,


def mutShrink(individual):
    """Replace a random branch by one of its arguments (``gp.py:854-882``)."""
    if len(individual) < 3 or individual.height <= 1:
        return individual,
    inner = [(i, node) for i, node in enumerate(individual[1:], 1)
             if isinstance(node, Primitive) and node.ret in node.args]
    if len(inner) != 0:
        index, prim = random.choice(inner)
        arg_idx = random.choice([i for i, t in enumerate(prim.args)
                                 if t == prim.ret])
        rindex = index + 1
        for _ in range(arg_idx + 1):
            rslice = individual.searchSubtree(rindex)
            subtree = individual[rslice]
            rindex += len(subtree)
        individual[individual.searchSubtree(index)] = subtree
    return individual,


def staticLimit(key, max_value):
    """Bloat control: an offspring over *max_value* is replaced by a random
    copy of one of the operator's inputs (reference ``gp.py:890-931``)."""
    def decorator(func):
        @wraps(func)
        def wrapper(*args, **kwargs):
            parents = [copy.deepcopy(ind) for ind in args]
            children = list(func(*args, **kwargs))
            for i, child in enumerate(children):
                if key(child) > max_value:
                    children[i] = random.choice(parents)
            return children
        return wrapper
    return decorator
