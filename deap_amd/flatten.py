"""Host flattener: ``PrimitiveTree`` → packed postfix bytecode for the HIP kernels.

Replaces, per individual, the reference's ``gp.compile`` (``deap/gp.py:462-487``:
``str(tree)`` → ``lambda`` → ``eval``).  Each tree is lowered to a short program
for one of two register machines executed by ``deap_amd/csrc/gpeval.hip``:

``F`` machine (fp64; symbolic regression and strongly-typed float/bool GP)
    One accumulator ``T`` (the value of the subtree just evaluated, K fitness
    cases per lane) plus a small operand stack ``R[0..D)`` in VGPRs.
``B`` machine (bit-sliced booleans; multiplexer / parity)
    Same shape; values are 32-case bit-planes.

Lowering rules
* Children are evaluated in Sethi–Ullman order (the child needing more
  registers first) so the stack depth stays ~log2(size); a non-commutative
  operator whose children were swapped is emitted in its *reversed* form
  (``rsub``, ``rdiv``, ``gt``).  Reordering is exact: primitives are pure and
  their arguments are evaluated eagerly (reference semantics), so the value
  does not depend on evaluation order.
* A terminal child is fused into its parent (``T = T op X[v]``/``T op c``).
* Argument-free subtrees are folded on the host by calling the primitive set's
  own Python callables — i.e. with exactly the reference's semantics
  (Python ints, ``protectedDiv``'s int 1, ``math.cos`` of glibc).  A folded
  subtree that raises makes the individual raise that exception.
* Trees higher than 200 raise ``SyntaxError``, like ``gp.compile`` on
  CPython 3.10 ("too many nested parentheses").

Word encoding (32 bit): ``op | depth << 8 | index << 16``; an F-machine
constant follows its instruction as two words (the f64 bits, low word first).
"""
import math
import os
import operator
from collections import namedtuple

import numpy as np


__all__ = ["Op", "Machine", "PsetSpec", "analyse_pset", "Flattener",
           "ProgramBatch", "MAX_COMPILE_HEIGHT"]

# CPython 3.10 tokenizer MAXLEVEL: 201 nested parentheses raise SyntaxError.
MAX_COMPILE_HEIGHT = 200
_EXACT_INT = 2 ** 53
# the exact-integer pass (gpe_load_exact_v) keeps ints on the device as sign
# + 1088-bit magnitude (GPE_XINT_WORDS uint32 words); programs with wider
# ints are evaluated by the library's host evaluator (unbounded ints)
XINT_BITS = 1088
XINT_WORDS = XINT_BITS // 32
_BOUND_CAP = 2 ** 1100         # bounds saturate here (they only meet < tests)


# GPE_NEG_PEEPHOLE=0 (A/B measurements): host-flattened programs keep every
# NEG (device lowering always folds them)
_NEG_PEEPHOLE = os.environ.get("GPE_NEG_PEEPHOLE", "1") != "0"


class ExactIntRangeError(ArithmeticError):
    """Raised only by the test twin of the device's exact-int interpreter
    (_lib.host_exact_eval) for an int past its 1088 bits; the evaluators
    never return it: the library evaluates such programs on the host with
    unbounded ints (the reference's Python ints)."""


class IntTable(object):
    """The exact pass's int constants: row r (the value of the program words'
    row index r) as little-endian 32-bit two's complement words
    ``words[off[r]:off[r + 1]]``, as few as hold the value and its sign."""

    def __init__(self, ints=None):
        vals = [0] * len(ints or ())
        for v, r in (ints or {}).items():
            vals[r] = v
        self.values = vals
        words, off = [], [0]
        for v in vals:
            n = v.bit_length() // 32 + 1         # room for the sign bit
            u = v & ((1 << (32 * n)) - 1)
            words.extend((u >> (32 * i)) & 0xFFFFFFFF for i in range(n))
            off.append(len(words))
        self.words = np.asarray(words, dtype=np.uint32)
        self.off = np.asarray(off, dtype=np.int64)

    def __len__(self):
        return len(self.values)


class Op:
    """Opcodes shared with ``gpeval.hip`` (keep in sync with ``gpe_op``)."""
    END = 0
    LDV = 1        # T = X[idx]
    LDC = 2        # T = const
    PUSH = 3       # R[d] = T
    PUSHV = 4      # R[d] = T; T = X[idx]
    PUSHC = 5      # R[d] = T; T = const
    # binary families: base + form, form 0 = stack R[d], 1 = var, 2 = const
    ADD = 8
    SUB = 11       # T = L - R  (left operand is the stack/var/const)
    RSUB = 14      # T = T - operand
    MUL = 17
    DIV = 20       # protectedDiv(operand, T)
    RDIV = 23      # protectedDiv(T, operand)
    LT = 26        # operand < T
    GT = 29        # T < operand      (lt with swapped children)
    EQ = 32
    AND = 35
    OR = 38
    XOR = 41
    NEG = 48
    SIN = 49
    COS = 50
    NOT = 51
    ITE = 52       # T = R[d] ? R[d+1] : T
    # numpy-semantics protected division (examples/gp/symbreg_numpy.py:
    # 28-36): q = l / r, then inf or nan -> 1
    NPDIV = 56     # npdiv(operand, T)
    RNPDIV = 59    # npdiv(T, operand)


_FORM_S, _FORM_V, _FORM_C = 0, 1, 2


class Machine:
    F = 0          # fp64 accumulator machine
    B = 1          # bit-sliced boolean machine


# error codes reported per individual (shared with the kernels)
ERR_NONE = 0
ERR_VALUE = 1          # math.sin/cos of +-inf  -> ValueError
ERR_OVERFLOW = 2       # (d)**2 overflow         -> OverflowError
ERR_SYNTAX = 3         # tree too deep for gp.compile
ERR_CONST = 4          # a folded constant subtree raised (see .const_exc)
ERR_NAMES = {ERR_VALUE: ValueError, ERR_OVERFLOW: OverflowError,
             ERR_SYNTAX: SyntaxError}


def _divides_small(fn):
    """A plain quotient for tiny nonzero divisors: rules out threshold
    protection such as ``l / r if abs(r) > 1e-6 else 1`` (gplearn-style),
    whose results the kernels' r == 0 test would not reproduce."""
    return (fn(1.0, 2.0 ** -1000) == 2.0 ** 1000
            and fn(1.0, 2.0 ** -40) == 2.0 ** 40
            and fn(3.0, -2.0 ** -23) == -3.0 * 2.0 ** 23
            and fn(1.0, 2.0 ** -9) == 512.0)


def _is_pdiv(fn):
    try:
        return (fn(6.0, 3.0) == 2.0 and fn(-3.0, 2.0) == -1.5
                and fn(1.0, 0.0) == 1 and fn(1.0, -0.0) == 1
                and fn(0.0, 0.0) == 1 and fn(7, 0) == 1 and fn(1, 2) == 0.5
                and math.isinf(fn(1e308, 1e-10)) and _divides_small(fn))
    except Exception:
        return False


def _is_np_pdiv(fn):
    """symbreg_numpy.py:28-36: numpy.divide with inf/nan mapped to 1."""
    try:
        with np.errstate(all="ignore"):
            return (fn(6.0, 3.0) == 2.0 and fn(1.0, 0.0) == 1
                    and fn(0.0, 0.0) == 1 and fn(1e308, 1e-10) == 1
                    and fn(-3.0, 2.0) == -1.5 and _divides_small(fn))
    except Exception:
        return False


def _is_ite(fn):
    try:
        return (fn(True, "a", "b") == "a" and fn(False, "a", "b") == "b"
                and fn(1, 2.0, 3.0) == 2.0 and fn(0, 2.0, 3.0) == 3.0)
    except Exception:
        return False


# callable → semantic name
_KNOWN = {operator.add: "add", operator.sub: "sub", operator.mul: "mul",
          operator.neg: "neg", math.sin: "sin", math.cos: "cos",
          operator.and_: "and", operator.or_: "or", operator.xor: "xor",
          operator.not_: "not", operator.lt: "lt", operator.eq: "eq",
          # numpy ufuncs of symbreg_numpy.py:39-45 (same IEEE arithmetic;
          # sin/cos of inf give nan instead of raising)
          np.add: "add", np.subtract: "sub", np.multiply: "mul",
          np.negative: "neg", np.sin: "npsin", np.cos: "npcos"}
TRIG = ("sin", "cos", "npsin", "npcos")

_F_BINARY = {"add": (Op.ADD, Op.ADD), "sub": (Op.SUB, Op.RSUB),
             "mul": (Op.MUL, Op.MUL), "pdiv": (Op.DIV, Op.RDIV),
             "lt": (Op.LT, Op.GT), "eq": (Op.EQ, Op.EQ),
             "and": (Op.AND, Op.AND), "or": (Op.OR, Op.OR),
             "npdiv": (Op.NPDIV, Op.RNPDIV)}
_F_UNARY = {"neg": Op.NEG, "sin": Op.SIN, "cos": Op.COS, "not": Op.NOT,
            "npsin": Op.SIN, "npcos": Op.COS}
_B_BINARY = {"and": (Op.AND, Op.AND), "or": (Op.OR, Op.OR),
             "xor": (Op.XOR, Op.XOR)}
_B_UNARY = {"not": Op.NOT}

PsetSpec = namedtuple("PsetSpec", "machine prim_ops arg_index has_trig")

# semantic name -> code of the native flattener (csrc/flatten_native.cpp)
_NATIVE_SEM = {"add": 0, "sub": 1, "mul": 2, "pdiv": 3, "neg": 4, "sin": 5,
               "cos": 6, "and": 7, "or": 8, "xor": 9, "not": 10, "lt": 11,
               "eq": 12, "ite": 13, "npdiv": 14, "npsin": 15, "npcos": 16}


def analyse_pset(pset, machine=None, adf_names=()):
    """Map every primitive of *pset* to kernel semantics.  Primitives named
    in *adf_names* are calls of automatically defined functions
    (``addADF``, gp.py:414-422) and are inlined by :class:`ADFFlattener`.

    Raises ``NotImplementedError`` for a primitive the kernels do not
    implement (the evaluator never falls back to the CPU)."""
    sem = {}
    adf_names = set(adf_names)
    for name, fn in pset.context.items():
        if name == "__builtins__" or not callable(fn) or name in adf_names:
            continue
        if fn in _KNOWN:
            sem[name] = _KNOWN[fn]
        elif _is_np_pdiv(fn):          # before pdiv: both map x/0 to 1
            sem[name] = "npdiv"
        elif _is_pdiv(fn):
            sem[name] = "pdiv"
        elif _is_ite(fn):
            sem[name] = "ite"
    prims = [p for plist in pset.primitives.values() for p in plist]
    names = {p.name for p in prims} - adf_names
    missing = sorted(n for n in names if n not in sem)
    if missing:
        raise NotImplementedError(
            "primitives without a GPU implementation: %s" % ", ".join(missing))
    used = {sem[n] for n in names}
    if machine is None:
        machine = Machine.B if used <= {"and", "or", "xor", "not", "ite"} \
            else Machine.F
    if machine == Machine.B and not used <= {"and", "or", "xor", "not",
                                              "ite"}:
        raise NotImplementedError("boolean machine cannot run %s"
                                  % sorted(used))
    if machine == Machine.F and "xor" in used:
        raise NotImplementedError("xor is only implemented on bit-planes")
    arg_index = {name: i for i, name in enumerate(pset.arguments)}
    prim_ops = {n: sem[n] for n in names}
    return PsetSpec(machine, prim_ops, arg_index, bool(used & set(TRIG)))


class _Const(object):
    __slots__ = ("value", "exc")

    def __init__(self, value, exc=None):
        self.value = value
        self.exc = exc


class ProgramBatch(object):
    """Packed programs for one ``gpe_eval`` call."""

    def __init__(self, code, offsets, depth, length, err, const_exc,
                 inexact):
        self.code = code            # uint32[n_words]
        self.offsets = offsets      # int64[n+1]
        self.depth = depth          # int32[n]  operand-stack slots needed
        # int64[n] reference node count (None: the differences of
        # `node_offsets`, formed on first use)
        self._length = length
        self.node_offsets = None
        self.err = err              # uint8[n]  compile-time error codes
        self.const_exc = const_exc  # {i: exception instance}
        # indices that may compute Python ints beyond 2**53 at run time:
        # candidates for the exact-integer pass (Flattener.exact_programs)
        self.inexact = inexact
        # {i: OverflowError} for inexact programs holding an int constant
        # past the float range, kept for the exact pass (which raises where
        # the reference converts it); a run without that pass (fp32, modes
        # it does not serve) raises this for the individual instead
        self.big_const = {}

    def __len__(self):
        return len(self.offsets) - 1

    @property
    def length(self):
        if self._length is None:
            self._length = np.diff(self.node_offsets)
        return self._length

    @length.setter
    def length(self, v):
        self._length = v

    def n_nodes(self):
        """The reference node count of all the batch's trees."""
        if self._length is None:
            return int(self.node_offsets[-1] - self.node_offsets[0])
        return int(self._length.sum())


def _too_deep(tree):
    """gp.compile of a tree over 200 levels: CPython 3.10 SyntaxError."""
    return len(tree) > MAX_COMPILE_HEIGHT and tree.height > MAX_COMPILE_HEIGHT


_INT_BINARY = ("add", "sub", "mul")


def _int_bounds(root):
    """Where a program's Python ints outgrow float64 (lower_core.h prim_ib,
    exactly).  A node's bound is the largest ``|value|`` over the cases
    where the value is a Python int (-1: never an int); per-case ints come
    from int constants and ``protectedDiv``'s int 1 (symbreg.py:29-33) and
    stay ints through add/sub/mul/neg.  Returns ``(needed, peak)``: needed if
    some primitive computes an int past 2**53 (add/sub/mul/neg), divides two
    ints one of which is past it, or compares one (Python rounds the exact
    ratio and compares exactly; a float64 would not); peak is the largest
    int bound in the program."""
    memo = {}
    need = False
    peak = 0
    todo = [(root, False)]
    while todo:
        rec, ready = todo.pop()
        key = id(rec)
        if key in memo:
            continue
        kind = rec[0]
        if kind == "v":
            memo[key] = -1
            continue
        if kind == "c":
            c = rec[1]
            v = c.value
            b = -1
            if c.exc is None and isinstance(v, int):     # bool: 0 / 1
                b = min(abs(int(v)), _BOUND_CAP)
                peak = max(peak, b)
            memo[key] = b
            continue
        if not ready:
            todo.append((rec, True))
            todo.extend((k, False) for k in rec[2])
            continue
        sem = rec[1]
        kb = [memo[id(k)] for k in rec[2]]
        if sem == "seq":
            b = kb[-1]
        elif sem in _INT_BINARY:
            if kb[0] < 0 or kb[1] < 0:
                b = -1
            else:
                b = min(kb[0] * kb[1] if sem == "mul" else kb[0] + kb[1],
                        _BOUND_CAP)
                need |= b > _EXACT_INT
        elif sem == "neg":
            b = kb[0]
            need |= b > _EXACT_INT
        elif sem == "pdiv":
            b = 1
            need |= kb[0] >= 0 and kb[1] >= 0 and max(kb) > _EXACT_INT
        elif sem in ("lt", "eq"):
            b = 1
            need |= max(kb) > _EXACT_INT
        elif sem in ("and", "or", "xor", "not"):
            b = 1
        elif sem == "ite":
            b = max(kb[1], kb[2])
        else:                              # sin/cos: floats; numpy semantics
            b = -1
        memo[key] = b
        peak = max(peak, b)
    return need, peak


def _exact_programs(fl, build, too_deep, length_of, trees):
    """Flattener.exact_programs for a lowering (*fl*, with *build*)."""
    index, keep = [], []
    for j, tree in enumerate(trees):
        if too_deep(tree):
            continue
        need, _ = _int_bounds(build(tree))
        if need:
            index.append(j)
            keep.append(tree)
    ints = {}
    batch = fl._lower(keep, build, length_of, too_deep, ints)
    return index, batch.code, batch.offsets, batch.depth, IntTable(ints), {}


class Flattener(object):
    """Lower trees of one primitive set (see module docstring)."""

    def __init__(self, pset, machine=None, trig_leaves=(), adf_call=None,
                 adf_names=()):
        self.pset = pset
        self.spec = analyse_pset(pset, machine, adf_names)
        self.machine = self.spec.machine
        ctx = pset.context
        self._fn = {n: ctx[n] for n in self.spec.prim_ops}
        # ADF primitive name -> callback(name, kid records) -> record
        self._adf_call = adf_call
        self._adf_names = frozenset(adf_names)
        # sin(ARGv)/cos(ARGv) leaves read device columns nv + v / 2 nv + v
        # (gpe_set_trig_leaves) for the argument indices listed here
        self.trig_leaves = frozenset(trig_leaves)
        self._nv = len(self.spec.arg_index)

    # ---------------------------------------------------------- analysis --
    def _build(self, tree, env=None, used=None):
        """Postfix pass: returns the root node record.

        Record: ``(kind, payload, children, need)`` with kind ``"v"`` (argument
        index), ``"c"`` (_Const) or ``"p"`` (semantic op name, or ``"seq"``:
        evaluate every child, keep the last).  With *env* (an ADF body), the
        argument terminals stand for the caller's argument records; the
        indices referenced are added to *used*."""
        args = self.spec.arg_index
        prim_ops = self.spec.prim_ops
        fns = self._fn
        leaves = self.trig_leaves
        stack = []
        for node in reversed(tree):
            arity = node.arity
            if arity == 0:
                # duck-typed on the reference's node protocol (arity, name,
                # value, conv_fct: gp.py:216-240) so trees built by deap.gp
                # itself flatten too
                if node.conv_fct is str and node.value in args:
                    if env is not None:
                        used.add(args[node.value])
                        stack.append(env[args[node.value]])
                    else:
                        stack.append(("v", args[node.value], None, 1))
                    continue
                value = node.value
                if node.conv_fct is str:          # named terminal
                    value = self.pset.context[node.value]
                stack.append(("c", _Const(value), None, 1))
                continue
            kids = [stack.pop() for _ in range(arity)]
            if node.name in self._adf_names:
                stack.append(self._adf_call(node.name, kids))
                continue
            sem = prim_ops[node.name]
            if leaves and sem in TRIG and \
                    kids[0][0] == "v" and kids[0][1] in leaves:
                col = (1 if sem in ("sin", "npsin") else 2) * self._nv \
                    + kids[0][1]
                stack.append(("v", col, None, 1))
                continue
            if all(k[0] == "c" for k in kids):
                stack.append(("c", self._fold(fns[node.name], kids), None, 1))
                continue
            stack.append(("p", sem, kids, self._need(sem, kids)))
        return stack[0]

    @staticmethod
    def _fold(fn, kids):
        for k in kids:
            if k[1].exc is not None:
                return _Const(None, k[1].exc)
        try:
            with np.errstate(all="ignore"):    # numpy ufuncs warn, not raise
                return _Const(fn(*[k[1].value for k in kids]))
        except Exception as exc:  # reference semantics: the call raises
            return _Const(None, exc)

    @staticmethod
    def _need(sem, kids):
        if sem == "seq":
            return max(k[3] for k in kids)
        if len(kids) == 1:
            return kids[0][3]
        if len(kids) == 3:
            return max(kids[0][3], 1 + kids[1][3], 2 + kids[2][3])
        left, right = kids
        if right[0] != "p":
            return left[3]
        if left[0] != "p":
            return right[3]
        nl, nr = left[3], right[3]
        return nl + 1 if nl == nr else max(nl, nr)

    # ---------------------------------------------------------- emission --
    def _emit(self, rec, d, out):
        """Append instructions leaving *rec*'s value in T; R[d..] is free.
        Returns the highest stack slot index + 1 used."""
        kind = rec[0]
        if kind == "v":
            out.append((Op.LDV, d, rec[1]))
            return d
        if kind == "c":
            out.append((Op.LDC, d, rec[1]))
            return d
        sem, kids = rec[1], rec[2]
        if sem == "seq":          # dead ADF arguments, then the body
            return max(self._emit(k, d, out) for k in kids)
        if len(kids) == 1:
            top = self._emit(kids[0], d, out)
            op = (_F_UNARY if self.machine == Machine.F else _B_UNARY)[sem]
            out.append((op, d, 0))
            return top
        if len(kids) == 3:        # if_then_else(cond, a, b)
            t0 = self._emit(kids[0], d, out)
            out.append((Op.PUSH, d, 0))
            t1 = self._emit(kids[1], d + 1, out)
            out.append((Op.PUSH, d + 1, 0))
            t2 = self._emit(kids[2], d + 2, out)
            out.append((Op.ITE, d, 0))
            return max(t0, t1, t2, d + 2)
        table = _F_BINARY if self.machine == Machine.F else _B_BINARY
        fwd, rev = table[sem]
        left, right = kids
        if right[0] != "p":                       # T = left; T = T op right
            top = self._emit(left, d, out)
            out.append(self._operand(rev, right, d))
            return top
        if left[0] != "p":                        # T = right; T = left op T
            top = self._emit(right, d, out)
            out.append(self._operand(fwd, left, d))
            return top
        if left[3] >= right[3]:
            t0 = self._emit(left, d, out)
            out.append((Op.PUSH, d, 0))
            t1 = self._emit(right, d + 1, out)
            out.append((fwd, d, None))                      # T = R[d] op T
            return max(t0, t1, d + 1)
        t0 = self._emit(right, d, out)
        out.append((Op.PUSH, d, 0))
        t1 = self._emit(left, d + 1, out)
        out.append((rev, d, None))                          # T = T op R[d]
        return max(t0, t1, d + 1)

    @staticmethod
    def _operand(op, leaf, d):
        if leaf[0] == "v":
            return (op + _FORM_V, d, leaf[1])
        return (op + _FORM_C, d, leaf[1])

    # ---------------------------------------------------------- encoding --
    def _encode(self, instrs, words, ints=None):
        F = self.machine == Machine.F
        n = len(instrs)
        i = 0
        # F machine: a NEG waits for the next instruction, which absorbs it
        # when it is an add or a sub (a + -T is a - T and a - -T is a + T,
        # exactly, signed zeros included), passes it on when it is a mul
        # (a * -T is -(a * T)); a second NEG cancels it (lower_core.h
        # Emitter, the same peephole).  Not in the exact pass's programs:
        # Python's int 0 has no sign (a = -0.0, T = 0: a + -T is 0.0, a - T
        # is -0.0), and that pass reproduces every value; the fitness never
        # sees a zero's sign (squared errors, protectedDiv's 1 for +-0)
        pneg = False
        while i < n:
            op, d, x = instrs[i]
            if F and op == Op.NEG and ints is None and _NEG_PEEPHOLE:
                pneg = not pneg
                i += 1
                continue
            if pneg:
                fam = op - Op.ADD
                if Op.ADD <= op < Op.RSUB:
                    op = op + 3 if fam < 3 else op - 3
                    pneg = False
                elif not Op.MUL <= op < Op.MUL + 3:    # a mul passes it on
                    words.append(Op.NEG)
                    pneg = False
            if op == Op.PUSH and i + 1 < n and instrs[i + 1][0] in (Op.LDV,
                                                                    Op.LDC):
                nop, _, nx = instrs[i + 1]
                op = Op.PUSHV if nop == Op.LDV else Op.PUSHC
                x = nx
                i += 1
            if op in (Op.LDC, Op.PUSHC) or (op >= Op.ADD and op < Op.NEG
                                             and (op - Op.ADD) % 3 == 2) \
                    or (op >= Op.NPDIV and (op - Op.NPDIV) % 3 == 2):
                row = None
                if ints is not None and isinstance(x.value, int):
                    key = int(x.value)          # True -> 1: the same int
                    if key not in ints:
                        ints[key] = len(ints)
                    row = ints[key]
                # an exact-pass int: index field 1, its table row in the
                # data words (no limit on the table's size)
                words.append(op | (d << 8) | ((row is not None) << 16) if F else
                             op | (d << 8) | (self._bmask(x) << 16))
                if F:
                    lo, hi = (row & 0xFFFFFFFF, row >> 32) if row is not None \
                        else self._f64_words(x)
                    words.append(lo)
                    words.append(hi)
            elif x is None:
                words.append(op | (d << 8))
            else:
                words.append(op | (d << 8) | (int(x) << 16))
            i += 1
        if pneg:
            words.append(Op.NEG)
        words.append(Op.END)

    @staticmethod
    def _f64_words(c):
        try:
            f = float(c.value)
        except OverflowError:       # an exact-pass int past the float range
            f = math.inf if c.value > 0 else -math.inf
        bits = np.float64(f).view(np.uint64)
        return int(bits) & 0xFFFFFFFF, int(bits) >> 32

    @staticmethod
    def _bmask(c):
        return 1 if c.value else 0

    # ------------------------------------------------------------ native --
    def _native_handle(self):
        """Tables for the native flattener (csrc/flatten_native.cpp): every
        shared node of the pset by identity and by name."""
        if getattr(self, "_nat", None) is not None:
            return self._nat
        from . import _flatnative
        args = self.spec.arg_index
        ids, entries, by_name, seen, eph = [], [], {}, set(), []

        def add(obj, entry):
            if id(obj) in seen:
                return
            seen.add(id(obj))
            by_name[obj.name] = len(entries)
            ids.append(id(obj))
            entries.append(entry)
        for plist in self.pset.primitives.values():
            for p in plist:
                add(p, (0, p.arity, _NATIVE_SEM[self.spec.prim_ops[p.name]],
                        0, None))
        for tlist in self.pset.terminals.values():
            for t in tlist:
                if isinstance(t, type):            # ephemeral class
                    eph.append(t)
                    continue
                if t.conv_fct is str and t.value in args:
                    add(t, (1, 0, 0, args[t.value], None))
                elif t.conv_fct is str:
                    add(t, (2, 0, 0, 0, self.pset.context[t.value]))
                else:
                    add(t, (2, 0, 0, 0, t.value))
        leaves = bytes(1 if v in self.trig_leaves else 0
                       for v in range(self._nv))
        # the `value` slot descriptor of the terminal class (fast reads of
        # ephemeral values); anything else falls back to getattr
        descr = None
        for klass in (eph[0].__mro__ if eph else ()):
            if "value" in klass.__dict__:
                descr = klass.__dict__["value"]
                break
        self._nat = (_flatnative.new(self.machine, self._nv, leaves, ids,
                                     entries, by_name, eph, descr),
                     (ids, entries, eph))
        return self._nat

    def read_codes(self, trees, start=0, stop=None):
        """The host half of device lowering: per node its pset entry (one
        byte, prefix order; 255 = an ephemeral whose value follows in
        ``evals``), for ``trees[start:stop]`` (read in place, no slice).
        Returns ``(codes, node_off, evals, eph_off)`` bytes, or None when
        the batch needs the host flattener (a tree the native reader
        declines or one that needs the interpreter)."""
        cap = self._native_handle()[0]
        from . import _flatnative
        return _flatnative.read_codes(cap, trees, int(start),
                                      -1 if stop is None else int(stop))

    def read_lower(self, trees, ends, lower_add, ctx, off, start=0):
        """read_codes and the library's gpe_lower_add as one pipeline
        (csrc/flatten_native.cpp read_lower): chunk k+1 is read while chunk
        k is staged and launched on a thread of its own.  The trees
        ``trees[start:ends[-1]]`` in chunks ending at *ends*.  *lower_add*
        and *ctx*: addresses of gpe_lower_add and of the context; *off*:
        int64 [n + 1] filled with their node offsets (from 0).  Returns 0,
        the lowering's error code, or None (a chunk needs the host
        flattener)."""
        cap = self._native_handle()[0]
        from . import _flatnative
        return _flatnative.read_lower(cap, trees, list(ends), int(lower_add),
                                      int(ctx), off, int(start))

    def lowering_tables(self):
        """(machine, nv, leaf bytes, entries bytes, n_entries) for
        gpe_set_lowering."""
        cap, (ids, entries, eph) = self._native_handle()
        from . import _flatnative
        leaves = bytes(1 if v in self.trig_leaves else 0 for v in range(self._nv))
        return (self.machine, self._nv, leaves, _flatnative.entries(cap),
                len(entries))

    def flatten(self, trees):
        """Lower *trees* into a :class:`ProgramBatch` (native flattener;
        trees it declines go through :meth:`flatten_py`)."""
        trees = list(trees)
        cap = self._native_handle()[0]
        from . import _flatnative
        (code, off, depth, length, err, inexact, declined,
         verr) = _flatnative.flatten(cap, trees)
        code = np.frombuffer(code, dtype=np.uint32)
        off = np.frombuffer(off, dtype=np.int64)
        depth = np.frombuffer(depth, dtype=np.int32).copy()
        length = np.frombuffer(length, dtype=np.int64).copy()
        err = np.frombuffer(err, dtype=np.uint8).copy()
        const_exc = {i: ValueError("math domain error") for i in verr}
        inexact = list(inexact)
        big_const = {}
        if declined:
            sub = self.flatten_py([trees[i] for i in declined])
            pieces, new_off, pos, last = [], [0], 0, 0
            fix = dict(zip(declined, range(len(declined))))
            for i in range(len(trees)):
                if i in fix:
                    j = fix[i]
                    seg = sub.code[sub.offsets[j]:sub.offsets[j + 1]]
                    depth[i] = sub.depth[j]
                    err[i] = sub.err[j]
                    if j in sub.const_exc:
                        const_exc[i] = sub.const_exc[j]
                    if j in sub.inexact:
                        inexact.append(i)
                    if j in sub.big_const:
                        big_const[i] = sub.big_const[j]
                else:
                    seg = code[off[i]:off[i + 1]]
                pieces.append(seg)
                pos += len(seg)
                new_off.append(pos)
            code = np.concatenate(pieces).astype(np.uint32)
            off = np.asarray(new_off, dtype=np.int64)
            inexact.sort()
        batch = ProgramBatch(code, off, depth, length, err, const_exc,
                             inexact)
        batch.big_const = big_const
        return batch

    def flatten_py(self, trees):
        """Lower *trees* into a :class:`ProgramBatch` (the Python
        specification of the lowering)."""
        return self._lower(trees, self._build, len, _too_deep)

    def _lower(self, trees, build, length_of, too_deep, ints=None):
        """*ints* (a dict): encode int constants for the exact-integer pass
        (their index + 1 in the word's index field, :meth:`exact_programs`)."""
        words = []
        offsets = np.zeros(len(trees) + 1, dtype=np.int64)
        depth = np.zeros(len(trees), dtype=np.int32)
        length = np.zeros(len(trees), dtype=np.int64)
        err = np.zeros(len(trees), dtype=np.uint8)
        const_exc = {}
        inexact = []
        big_const = {}
        F = self.machine == Machine.F
        for i, tree in enumerate(trees):
            offsets[i] = len(words)
            length[i] = length_of(tree)
            if too_deep(tree):
                err[i] = ERR_SYNTAX
                words.append(Op.END)
                continue
            root = build(tree)
            if root[0] == "c":
                c = root[1]
                if c.exc is not None:
                    err[i] = ERR_CONST
                    const_exc[i] = c.exc
                    words.append(Op.END)
                    continue
            instrs = []
            depth[i] = self._emit(root, 0, instrs)
            need = F and self._python_ints and _int_bounds(root)[0]
            if F and not self._check_consts(instrs, i, const_exc, err, need,
                                            big_const):
                del words[offsets[i]:]
                words.append(Op.END)
                continue
            if need:
                inexact.append(i)
            self._encode(instrs, words, ints)
        offsets[-1] = len(words)
        code = np.asarray(words, dtype=np.uint32)
        batch = ProgramBatch(code, offsets, depth, length, err, const_exc,
                             inexact)
        batch.big_const = big_const
        return batch

    @staticmethod
    def _check_consts(instrs, i, const_exc, err, exact=False, kept=None):
        """Constants must convert to f64 the way Python's mixed int/float
        arithmetic converts them; a raising fold raises for the individual.
        With *exact* (the program goes to the exact-integer pass) an int
        constant past the float range that the pass holds is kept: the pass
        raises OverflowError where the reference converts it, and nowhere
        else (an int compared or combined with ints); its OverflowError goes
        to *kept* for a run without the pass."""
        for op, _, x in instrs:
            if isinstance(x, _Const):
                if x.exc is not None:
                    err[i] = ERR_CONST
                    const_exc[i] = x.exc
                    return False
                v = x.value
                if isinstance(v, int) and not isinstance(v, bool) \
                        and abs(v) > _EXACT_INT:
                    try:
                        float(v)
                    except OverflowError as exc:
                        if exact:
                            if kept is not None:
                                kept.setdefault(i, exc)
                            continue
                        err[i] = ERR_CONST
                        const_exc[i] = exc
                        return False
        return True

    @property
    def _python_ints(self):
        """Python-number semantics (not the numpy example's arrays, where
        ints never survive an operation)."""
        return not any(s in ("npdiv", "npsin", "npcos")
                       for s in self.spec.prim_ops.values())

    def exact_programs(self, trees):
        """The exact-integer pass's programs for *trees* (those a batch
        listed in ``inexact``): ``(index, code, offsets, depth, ints,
        refused)`` where *index* lists the trees that need the pass,
        *code*/*offsets*/*depth* their programs — the usual words, with every
        int constant's index field 1 and its row of *ints* (an
        :class:`IntTable`, any number of rows of any width) in its data
        words — and *refused* is empty (kept for callers: no tree is
        refused)."""
        return _exact_programs(self, self._build, _too_deep, len, trees)


class ADFFlattener(object):
    """Lowering of automatically-defined-function individuals
    (``gp.compileADF``, gp.py:490-513; ``examples/gp/adf_symbreg.py``).

    An individual is ``[main, adf_1, ..., adf_k]`` and *psets* the matching
    primitive sets, in compileADF's order.  compileADF turns every ADF tree
    into a Python function whose arguments are evaluated eagerly by the
    caller; here each call is inlined: the body of the called ADF tree is
    built with its argument terminals standing for the caller's argument
    records (a value shared by all its uses), recursively for ADFs that
    call ADFs.  Arguments the body never reads are still evaluated first
    (a ``seq`` record) when they could raise, as the eager call would."""

    def __init__(self, psets, machine=None):
        self.psets = list(psets)
        self.names = [p.name for p in self.psets[1:]]
        self._index = {n: i + 1 for i, n in enumerate(self.names)}
        self._fl = [Flattener(p, machine, adf_call=self._call,
                              adf_names=self.names) for p in self.psets]
        machines = {f.machine for f in self._fl}
        if len(machines) != 1:
            raise NotImplementedError("ADF primitive sets need one machine")
        self.machine = self._fl[0].machine
        self.spec = self._fl[0].spec
        self.trig_leaves = frozenset()
        self._ind = None

    def _call(self, name, kids):
        k = self._index[name]
        used = set()
        body = self._fl[k]._build(self._ind[k], env=kids, used=used)
        dead = [r for i, r in enumerate(kids) if i not in used and
                (r[0] == "p" or (r[0] == "c" and r[1].exc is not None))]
        if not dead:
            return body
        parts = dead + [body]
        return ("p", "seq", parts, max(r[3] for r in parts))

    def _build(self, ind):
        self._ind = ind
        try:
            return self._fl[0]._build(ind[0])
        finally:
            self._ind = None

    def flatten(self, individuals):
        """Lower ``[main, adf...]`` individuals into a :class:`ProgramBatch`
        (``length`` = total node count of the individual's trees)."""
        return self._fl[0]._lower(
            list(individuals), self._build,
            lambda ind: sum(len(t) for t in ind),
            lambda ind: any(_too_deep(t) for t in ind))

    flatten_py = flatten

    def exact_programs(self, individuals):
        """:meth:`Flattener.exact_programs` for ADF individuals."""
        return _exact_programs(
            self._fl[0], self._build,
            lambda ind: any(_too_deep(t) for t in ind),
            lambda ind: sum(len(t) for t in ind), list(individuals))
