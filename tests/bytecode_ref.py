"""Test helper: numpy interpreter of the flattened bytecode.

Mirrors the kernels' semantics (deap_amd/csrc/gpeval.hip) on the CPU so the
flattener can be checked against the oracle without a GPU.  Not product code.
"""
import math

import numpy as np

from deap_amd.flatten import Op

_FAMS = {Op.ADD: "add", Op.SUB: "sub", Op.RSUB: "rsub", Op.MUL: "mul",
         Op.DIV: "div", Op.RDIV: "rdiv", Op.LT: "lt", Op.GT: "gt",
         Op.EQ: "eq", Op.AND: "and", Op.OR: "or", Op.XOR: "xor",
         Op.NPDIV: "npdiv", Op.RNPDIV: "rnpdiv"}


def _f64(lo, hi):
    return np.array([int(lo) | (int(hi) << 32)], dtype=np.uint64).view(
        np.float64)[0]


def _fbin(name, a, b):
    with np.errstate(all="ignore"):
        if name == "add":
            return a + b
        if name == "sub":
            return a - b
        if name == "rsub":
            return b - a
        if name == "mul":
            return a * b
        if name == "div":
            return np.where(b == 0.0, 1.0, a / np.where(b == 0.0, 1.0, b))
        if name == "rdiv":
            return np.where(a == 0.0, 1.0, b / np.where(a == 0.0, 1.0, a))
        if name == "npdiv":                     # symbreg_numpy.py:28-36
            q = np.divide(a, b)
            return np.where(np.isfinite(q), q, 1.0)
        if name == "rnpdiv":
            q = np.divide(b, a)
            return np.where(np.isfinite(q), q, 1.0)
        if name == "lt":
            return (a < b).astype(np.float64)
        if name == "gt":
            return (b < a).astype(np.float64)
        if name == "eq":
            return (a == b).astype(np.float64)
        if name == "and":
            return ((a != 0) & (b != 0)).astype(np.float64)
        if name == "or":
            return ((a != 0) | (b != 0)).astype(np.float64)
    raise KeyError(name)


def run_f(code, X):
    """Returns (T, valueerror_mask) for one F program over all cases."""
    n = X.shape[1]
    T = np.zeros(n)
    R = {}
    verr = np.zeros(n, dtype=bool)
    pc = 0
    while True:
        w = int(code[pc]); pc += 1
        op, d, x = w & 0xff, (w >> 8) & 0xff, w >> 16
        if op == Op.END:
            return T, verr
        const = None
        takes_const = op in (Op.LDC, Op.PUSHC) or (
            Op.ADD <= op < Op.NEG and (op - Op.ADD) % 3 == 2) or (
            op >= Op.NPDIV and (op - Op.NPDIV) % 3 == 2)
        if takes_const:
            const = _f64(code[pc], code[pc + 1]); pc += 2
        if op == Op.LDV:
            T = X[x].copy()
        elif op == Op.LDC:
            T = np.full(n, const)
        elif op == Op.PUSH:
            R[d] = T
        elif op == Op.PUSHV:
            R[d] = T; T = X[x].copy()
        elif op == Op.PUSHC:
            R[d] = T; T = np.full(n, const)
        elif Op.ADD <= op < Op.NEG or op >= Op.NPDIV:
            b0 = Op.NPDIV if op >= Op.NPDIV else Op.ADD
            base = b0 + 3 * ((op - b0) // 3)
            form = (op - b0) % 3
            a = R[d] if form == 0 else (X[x] if form == 1 else const)
            T = _fbin(_FAMS[base], a, T)
        elif op == Op.NEG:
            T = -T
        elif op in (Op.SIN, Op.COS):
            verr |= np.isinf(T)
            fn = math.sin if op == Op.SIN else math.cos
            T = np.array([fn(v) if math.isfinite(v) else math.nan
                          for v in T.tolist()])
        elif op == Op.NOT:
            T = (T == 0).astype(np.float64)
        elif op == Op.ITE:
            T = np.where(R[d] != 0, R[d + 1], T)
        else:
            raise ValueError(op)


def run_b(code, planes):
    """Bit-plane program → uint32 word array."""
    nw = planes.shape[1]
    T = np.zeros(nw, dtype=np.uint32)
    R = {}
    full = np.uint32(0xFFFFFFFF)
    pc = 0
    while True:
        w = int(code[pc]); pc += 1
        op, d, x = w & 0xff, (w >> 8) & 0xff, w >> 16
        if op == Op.END:
            return T
        cm = np.full(nw, full if x else np.uint32(0), dtype=np.uint32)
        if op == Op.LDV:
            T = planes[x].copy()
        elif op == Op.LDC:
            T = cm
        elif op == Op.PUSH:
            R[d] = T
        elif op == Op.PUSHV:
            R[d] = T; T = planes[x].copy()
        elif op == Op.PUSHC:
            R[d] = T; T = cm
        elif Op.ADD <= op < Op.NEG or op >= Op.NPDIV:
            b0 = Op.NPDIV if op >= Op.NPDIV else Op.ADD
            base = b0 + 3 * ((op - b0) // 3)
            form = (op - b0) % 3
            a = R[d] if form == 0 else (planes[x] if form == 1 else cm)
            name = _FAMS[base]
            T = {"and": a & T, "or": a | T, "xor": a ^ T}[name]
        elif op == Op.NOT:
            T = ~T
        elif op == Op.ITE:
            T = (R[d] & R[d + 1]) | (~R[d] & T)
        else:
            raise ValueError(op)


def np_sse_from_T(T, values):
    """Mirror of SymbRegNumpySSE: per-case (T - values)**2, then the
    library's host twin of its numpy-order row sum."""
    from deap_amd import _lib
    with np.errstate(over="ignore", invalid="ignore"):
        sq = (T - values) * (T - values)
    return float(_lib.host_np_sum(sq)[0])


def mse_from_T(T, verr, terms):
    """Mirror of the MSE epilogue: returns fitness or exception name."""
    d = T.copy()
    for t in terms:
        d = d - t
    with np.errstate(over="ignore", invalid="ignore"):
        sq = d * d
    ovf = np.isfinite(d) & np.isinf(sq)
    err = np.where(verr, 1, np.where(ovf, 2, 0))
    bad = np.nonzero(err)[0]
    if len(bad):
        return "ValueError" if err[bad[0]] == 1 else "OverflowError"
    total = math.fsum(sq.tolist())
    return total / len(T)
