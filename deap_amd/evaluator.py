"""GPU population evaluator — the drop-in behind ``toolbox.map``/``evaluate``.

Reference hot path (chris-chambers/deap):

    toolbox.register("evaluate", evalSymbReg, points=...)   examples/gp/symbreg.py:63
    fitnesses = toolbox.map(toolbox.evaluate, invalid_ind)   deap/algorithms.py:172
      evalSymbReg: func = gp.compile(ind, pset)              deap/gp.py:462-487
                   math.fsum((func(x) - ...)**2 ...) / n     symbreg.py:55-61

Drop-in replacement (the EA loop, PrimitiveSet and PrimitiveTree unchanged):

    ev = GPUEvaluator(pset, SymbRegMSE.quartic())
    toolbox.register("evaluate", ev)
    toolbox.register("map", gpu_map)

``gpu_map(func, individuals)`` recognises a (``functools.partial``-wrapped)
:class:`GPUEvaluator`, flattens all individuals (:mod:`deap_amd.flatten`),
evaluates them in one call of the HIP library and returns the fitness tuples
in order.  Any other function goes to the builtin ``map`` — exactly the
reference's default (``deap/base.py:50``).  Like the reference's lazy ``map``
consumed by ``zip`` (``algorithms.py:173``), the result iterator yields the
individuals before the first failing one and then raises that individual's
exception (``ValueError`` from ``math.sin/cos(inf)``, ``OverflowError`` from
``d**2`` or ``fsum``, ``SyntaxError`` for trees over 200 levels, or whatever a
constant subtree raised).
"""
import math
import os
import time
import warnings
from functools import partial

import numpy as np

from . import _lib
from .flatten import (ADFFlattener, ERR_CONST, ERR_SYNTAX, Flattener,
                      Machine, ProgramBatch)


def _tuples1(values, as_int):
    """``[(v,), ...]`` for a float64 array (hit counts as ints), built by
    the native module in one pass."""
    from . import _flatnative
    return _flatnative.tuples1(np.ascontiguousarray(values, dtype=np.float64),
                               as_int)


__all__ = ["SymbRegMSE", "SymbRegNumpySSE", "SymbRegSumSSE",
           "SymbRegCaseErrors", "BooleanHits",
           "TypedBoolHits", "GPUEvaluator", "gpu_map", "pack_bitplanes"]


def _case_error(err):
    """The exception of a program's first erroring case (out_err's type)."""
    kind = int(err) & 3
    if kind == _lib.GPE_ERR_VALUE:
        return ValueError("math domain error")
    if kind == _lib.GPE_ERR_OVERFLOW:
        return OverflowError(34, "Numerical result out of range")
    # the device exact pass's range end (GPE_ERR_XINT_RANGE) never reaches
    # the caller: the library re-runs such programs on its host evaluator.
    # One that leaks is a library bug, not the reference's OverflowError
    raise _lib.GpeError("internal: per-case error kind %d (first error word "
                        "0x%x) reached the evaluator" % (kind, int(err)))


# --------------------------------------------------------- fitness specs --
class SymbRegMSE(object):
    """``(math.fsum((f(*row) - t0 - t1 - ...)**2 for each case) / n,)``.

    ``X``: float64 ``[n_vars, n_cases]``; ``terms``: float64
    ``[n_terms, n_cases]`` subtracted left to right (symbreg.py:60)."""
    machine = Machine.F
    mode = _lib.GPE_MODE_MSE

    def __init__(self, X, terms):
        self.X = np.ascontiguousarray(X, dtype=np.float64)
        if self.X.ndim == 1:
            self.X = self.X[None, :]
        t = np.ascontiguousarray(terms, dtype=np.float64)
        self.terms = t[None, :] if t.ndim == 1 else t
        self.n_cases = self.X.shape[1]
        assert self.terms.shape[1] == self.n_cases

    @classmethod
    def quartic(cls):
        """symbreg.py's ``x**4 + x**3 + x**2 + x`` on ``x/10.``, x in
        [-10, 10) — terms computed with Python ``**`` like the reference."""
        from .datasets import symbreg_points
        X, T = symbreg_points()
        return cls(X, T)

    def upload(self, ctx):
        ctx.set_cases(_lib.GPE_MACHINE_F, self.X, self.terms)

    def finish(self, i, hi, lo, err, flags):
        if err != _lib.GPE_NO_ERROR:
            return _case_error(err)
        sse = float(hi) + float(lo)
        if math.isinf(sse) and not (flags & _lib.GPE_FLAG_NONFINITE_TERM):
            return OverflowError("intermediate overflow in fsum")
        return (sse / self.n_cases,)

    def finish_all(self, hi, lo, err, flags):
        """:meth:`finish` for a whole batch (vectorised; the same IEEE
        operations, per-individual only where an exception is possible)."""
        sse = hi + lo
        with np.errstate(all="ignore"):
            out = _tuples1(sse / self.n_cases, False)          # 1-tuples, in C
        bad = (err != np.uint64(_lib.GPE_NO_ERROR)) | (
            np.isinf(sse) & ((flags & _lib.GPE_FLAG_NONFINITE_TERM) == 0))
        for i in np.flatnonzero(bad).tolist():
            out[i] = self.finish(i, hi[i], lo[i], err[i], flags[i])
        return out


class SymbRegNumpySSE(SymbRegMSE):
    """``(numpy.sum((func(samples) - values)**2),)`` — the vectorised
    evaluation of ``examples/gp/symbreg_numpy.py:62-68``.

    numpy semantics throughout: ``numpy.sin/cos(+-inf)`` is nan (no
    ``ValueError``), ``**2`` of a large finite value is inf (no
    ``OverflowError``), the protected division of ``symbreg_numpy.py:28-36``
    maps inf/nan quotients to 1 (``Op.NPDIV``), and the sum is not divided
    by n.  The device writes every squared term and sums each program's row
    in numpy.sum's own order (GPE_MODE_SSE_NUMPY: pairwise blocks of 128
    inside 8192-element chunks), so the sum is bit-identical to numpy's
    for identical terms; nan and inf propagate as they do there."""
    mode = _lib.GPE_MODE_SSE_NUMPY
    outputs = ("hi",)            # what finish_all reads (gpe_run copies)

    @classmethod
    def linspace(cls, n=10000):
        """The reference example's ``samples``/``values``."""
        from .datasets import symbreg_numpy_points
        X, V = symbreg_numpy_points(n)
        return cls(X, V)

    def finish(self, i, hi, lo, err, flags):
        return (float(hi),)

    def finish_all(self, hi, lo, err, flags):
        return _tuples1(hi, False)


class SymbRegSumSSE(SymbRegMSE):
    """``(sum((f(x) - target)**2 for each case),)`` with Python's builtin
    ``sum`` (left to right from 0, no division) — the evaluation of
    ``examples/gp/adf_symbreg.py:117-125``.  Exceptions as in
    :class:`SymbRegMSE` (``math.sin/cos(inf)``, ``d**2`` overflow); an
    overflowing sum is ``inf`` (no ``fsum`` error).  The device sums each
    program's terms in the same order (GPE_MODE_SSE_SEQ), bit for bit."""
    mode = _lib.GPE_MODE_SSE_SEQ

    @classmethod
    def adf_quartic(cls):
        from .datasets import adf_symbreg_points
        X, T = adf_symbreg_points()
        return cls(X, T)

    def finish(self, i, hi, lo, err, flags):
        if err != _lib.GPE_NO_ERROR:
            return SymbRegMSE.finish(self, i, hi, lo, err, flags)
        return (float(hi),)

    def finish_all(self, hi, lo, err, flags):
        out = _tuples1(hi, False)
        for i in np.flatnonzero(err != np.uint64(_lib.GPE_NO_ERROR)).tolist():
            out[i] = self.finish(i, hi[i], lo[i], err[i], flags[i])
        return out


class SymbRegCaseErrors(SymbRegMSE):
    """``tuple((f(*row) - t0 - ...)**2 for each case)`` — one fitness value
    per case, for lexicase selection (reference ``selLexicase`` and its
    epsilon variants, ``deap/tools/selection.py:214-320``, read
    ``fitness.values[case]``; the individual's weights are one per case).
    The device writes the per-case terms of the same reduction
    (``gpe_run_cases``)."""
    per_case = True

    def finish(self, i, hi, lo, err, flags, cases=None):
        if err != _lib.GPE_NO_ERROR:
            return SymbRegMSE.finish(self, i, hi, lo, err, flags)
        return tuple(cases.tolist())


def pack_bitplanes(bits):
    """``bits[n_rows, n_cases]`` in {0,1} → ``uint32[n_rows, ceil(n/32)]``,
    case c at bit c % 32 of word c // 32."""
    bits = np.asarray(bits, dtype=np.uint8)
    if bits.ndim == 1:
        bits = bits[None, :]
    n_rows, n = bits.shape
    n_words = (n + 31) // 32
    padded = np.zeros((n_rows, n_words * 32), dtype=np.uint64)
    padded[:, :n] = bits
    weights = (np.uint64(1) << np.arange(32, dtype=np.uint64))
    words = (padded.reshape(n_rows, n_words, 32) * weights).sum(axis=2)
    return words.astype(np.uint32)


class BooleanHits(object):
    """``(sum(func(*in_) == out for in_, out in zip(inputs, outputs)),)``
    (multiplexer.py:75, parity.py:68) on 0/1 inputs, bit-sliced."""
    machine = Machine.B
    mode = _lib.GPE_MODE_HITS_BITS
    outputs = ("hi",)

    def __init__(self, inputs, outputs):
        ins = np.asarray(inputs)
        outs = np.asarray(outputs)
        if ins.ndim != 2 or outs.shape != (ins.shape[1],):
            raise ValueError("inputs must be [n_vars, n_cases], outputs "
                             "[n_cases]")
        if not (np.isin(ins, (0, 1)).all() and np.isin(outs, (0, 1)).all()):
            raise NotImplementedError("bit-sliced evaluation needs 0/1 data")
        self.n_cases = ins.shape[1]
        self.planes = pack_bitplanes(ins)
        self.out_plane = pack_bitplanes(outs)[0]

    @classmethod
    def from_rows(cls, inputs, outputs):
        """Reference layout: ``inputs[case][var]``, ``outputs[case]``."""
        return cls(np.asarray(inputs).T, np.asarray(outputs))

    def upload(self, ctx):
        ctx.set_bitplanes(self.planes, self.out_plane, self.n_cases)

    def finish(self, i, hi, lo, err, flags):
        return (int(hi),)

    def finish_all(self, hi, lo, err, flags):
        return _tuples1(hi, True)


class TypedBoolHits(object):
    """``(sum(bool(func(*row)) is bool(label) for row, label ...),)``
    (spambase.py:86) evaluated on every row."""
    machine = Machine.F
    mode = _lib.GPE_MODE_HITS_BOOL
    outputs = ("hi", "err")
    # with no exact-integer pass and no sin/cos (ValueError) no case can
    # error: the counts alone
    outputs_plain = ("hi",)

    def __init__(self, X, labels):
        self.X = np.ascontiguousarray(X, dtype=np.float64)
        self.labels = (np.asarray(labels) != 0).astype(np.float64)[None, :]
        self.n_cases = self.X.shape[1]

    def upload(self, ctx):
        ctx.set_cases(_lib.GPE_MACHINE_F, self.X, self.labels)

    def finish(self, i, hi, lo, err, flags):
        # (errors only from the exact-integer pass: float(int) overflow)
        if err != _lib.GPE_NO_ERROR:
            return _case_error(err)
        return (int(hi),)

    def finish_all(self, hi, lo, err, flags):
        out = _tuples1(hi, True)
        if err is not None:
            for i in np.flatnonzero(err != np.uint64(_lib.GPE_NO_ERROR)).tolist():
                out[i] = _case_error(err[i])
        return out


# ------------------------------------------------------------- evaluator --
def trig_leaf_columns(pset_spec, spec, precision="fp64"):
    """Argument indices whose sin/cos leaves may be read from device columns:
    an F-machine spec whose case matrix holds one row per pset argument, and
    a finite column (math.sin/cos(+-inf) raises, so such leaves stay in the
    program where the error is reported at its first case) — in fp32 mode
    finite after the float cast the fp32 machine applies."""
    X = getattr(spec, "X", None)
    if not pset_spec.has_trig or spec.machine != Machine.F or X is None \
            or X.shape[0] != len(pset_spec.arg_index):
        return ()
    if precision == "fp32":
        with np.errstate(over="ignore"):
            X = X.astype(np.float32)
    return tuple(int(v) for v in np.flatnonzero(np.isfinite(X).all(axis=1)))


def _default_device():
    return int(os.environ.get("LOCAL_RANK", "0"))


class GPUEvaluator(object):
    """Evaluates populations of one primitive set on one fitness spec.

    Calling it on a single individual evaluates a batch of one (the
    reference's direct ``toolbox.evaluate(ind)`` calls); :func:`gpu_map`
    routes whole populations through :meth:`map`.

    *pset* may be a list of primitive sets ``[main, adf_1, ...]`` — the
    ``psets`` of ``gp.compileADF`` (gp.py:490-513) — for individuals that
    are lists of trees (``examples/gp/adf_symbreg.py``).
    """

    def __init__(self, pset, spec, device=None, machine=None,
                 trig_leaves=True, precision="fp64"):
        """*precision* ``"fp64"`` (default) matches the reference (1e-12
        relative MSE); ``"fp32"`` evaluates the trees in single precision
        for throughput, with the agreement DESIGN.md §4 states."""
        if precision not in ("fp64", "fp32"):
            raise ValueError("precision must be 'fp64' or 'fp32'")
        self.pset = pset
        self.spec = spec
        self.precision = precision
        machine = machine if machine is not None else spec.machine
        adf = isinstance(pset, (list, tuple))
        self.flattener = ADFFlattener(pset, machine) if adf else \
            Flattener(pset, machine)
        if self.flattener.machine != spec.machine:
            raise ValueError("fitness spec and primitive set need different "
                             "machines")
        self.ctx = _lib.Context(_default_device() if device is None
                                else device)
        spec.upload(self.ctx)
        if precision == "fp32":
            if spec.machine != Machine.F:
                raise ValueError("fp32 mode applies to the F machine only")
            self.ctx.set_precision(_lib.GPE_PREC_F32)
        # sin/cos of a bare argument: evaluated once per case on the device
        # (same function, same value) and read by every program
        leaves = trig_leaf_columns(self.flattener.spec, spec, precision) \
            if trig_leaves and not adf else ()
        if leaves:
            self.ctx.set_trig_leaves(True)
            self.flattener = Flattener(pset, machine, trig_leaves=leaves)
        self.stats = {"calls": 0, "individuals": 0, "node_evals": 0,
                      "flatten_s": 0.0, "device_s": 0.0, "kernel_ms": 0.0,
                      "device_lowered": 0}
        self._warned_inexact = False
        self._exact_flattener = None
        # device lowering (gpe_lower_programs): the host only reads each
        # node's pset entry; the register-machine words are built on the GPU
        self.device_lowering = not adf and \
            os.environ.get("GPE_DEVICE_LOWERING", "1") != "0"
        self._lowering_set = False
        # output arrays reused across evaluate calls (_lib.ResultBuffers)
        self._run_out = _lib.ResultBuffers()
        self._lw_out = _lib.LoweringBuffers()
        # the node offsets of a chunked lowering, reused when the batch
        # does not outlive the next lowering (keep=False: evaluate)
        self._lw_off = np.zeros(0, dtype=np.int64)
        # trees per chunk of a chunked device lowering (populations larger
        # than this are read and lowered in overlapping chunks)
        self.lower_chunk = int(os.environ.get("GPE_LOWER_CHUNK", 1 << 18))

    # the evaluator is used as toolbox.evaluate
    def __call__(self, individual):
        res = self.evaluate([individual])[0]
        if isinstance(res, BaseException):
            raise res
        return res

    def flatten(self, individuals):
        t0 = time.perf_counter()
        batch = self.flattener.flatten(individuals)
        self.stats["flatten_s"] += time.perf_counter() - t0
        self._warn_inexact(batch)
        return batch

    def lower_on_device(self, individuals, keep=True, lo=0, hi=None):
        """Read the trees' node codes on the host and lower them into the
        context's program buffers on the GPU.  Returns a :class:`ProgramBatch`
        without host words (``code`` None, already loaded), or None when the
        batch needs the host flattener (a node the native reader declines, a
        constant fold only Python can do, a pset of 255+ entries).  *keep*
        False: the batch is used only until the next lowering (its arrays
        stay in the evaluator's reused buffers).  *lo*, *hi*: lower only
        ``individuals[lo:hi]`` (read in place, no slice)."""
        hi = len(individuals) if hi is None else hi
        n = hi - lo
        if n > self.lower_chunk:
            return self._lower_chunked(individuals, keep, lo, hi)
        t0 = time.perf_counter()
        r = self.flattener.read_codes(individuals, lo, hi)
        self.stats["flatten_s"] += time.perf_counter() - t0
        if r is None:
            return None
        t0 = time.perf_counter()
        self._set_lowering()
        codes, node_off, evals, eph_off = r
        depth, err, status = self.ctx.lower_programs(codes, node_off, evals,
                                                     eph_off, out=self._lw_out)
        self.stats["device_s"] += time.perf_counter() - t0
        off = np.frombuffer(node_off, dtype=np.int64)
        return self._lowered_batch(off, depth, err, status, keep)

    def _set_lowering(self):
        if not self._lowering_set:
            self.ctx.set_lowering(*self.flattener.lowering_tables())
            self._lowering_set = True

    @staticmethod
    def _chunk_bounds(n, chunk, tail=None):
        """Chunk ends of a chunked lowering: equal chunks of at most
        ``chunk`` trees; with *tail*, the last ones halving (chunk / 2,
        chunk / 4, ... down to ``tail``).  Halving was meant to leave little
        device work after the host's last read, but each lower_trees launch
        has a ~0.4 ms floor (one wave lowering its 64 trees through
        dependent scratch accesses), so the small chunks cost more than they
        saved (C3 at pop 1M, same box: 9.4-10.9 ms without, 11.5-13.8 with
        a 2^14 tail).  ``GPE_LOWER_TAIL=N`` (N >= 1024) restores a tail."""
        env = os.environ.get("GPE_LOWER_TAIL", "")
        if tail is None and env.isdigit() and int(env) >= 1024:
            tail = int(env)
        halves = []
        c = chunk // 2 if tail else 0
        while tail and c >= tail and sum(halves) + c < n // 2:
            halves.append(c)
            c //= 2
        head = n - sum(halves)
        k = -(-head // chunk)
        ends = [head * (i + 1) // k for i in range(k)]
        for h in halves:
            ends.append(ends[-1] + h)
        return ends

    def _lower_chunked(self, individuals, keep=True, lo=0, hi=None):
        """lower_on_device in chunks of ``lower_chunk`` trees: the device
        uploads and lowers chunk i (gpe_lower_add, asynchronous) while the
        host reads chunk i + 1 (read_codes in place, no slices)."""
        hi = len(individuals) if hi is None else hi
        n = hi - lo
        self._set_lowering()
        if keep:
            off = np.empty(n + 1, dtype=np.int64)
        else:
            # (a fresh 8 MB array per call at pop 1M is fresh pages: their
            # first-touch faults and the unmapping)
            if len(self._lw_off) < n + 1:
                self._lw_off = np.empty(n + 1, dtype=np.int64)
            off = self._lw_off[:n + 1]
        off[0] = 0
        self.ctx.lower_begin(n, out=self._lw_out)
        ends = [lo + e for e in self._chunk_bounds(n, self.lower_chunk)]
        if os.environ.get("GPE_READ_LOWER", "1") != "0":
            # the pipeline in native code: the next chunk's read overlaps
            # the previous one's staging and launch (gpe_lower_add)
            t0 = time.perf_counter()
            rc = self.flattener.read_lower(individuals, ends,
                                           self.ctx.lower_add_addr(),
                                           self.ctx.handle_addr(), off, lo)
            self.stats["flatten_s"] += time.perf_counter() - t0
            if rc is None:
                return None            # (the next lowering or load resets)
            self.ctx.check_rc(rc, "gpe_lower_add")
            t0 = time.perf_counter()
            depth, err, status = self.ctx.lower_end(out=self._lw_out)
            self.stats["device_s"] += time.perf_counter() - t0
            return self._lowered_batch(off, depth, err, status, keep)
        a = lo
        for b in ends:
            t0 = time.perf_counter()
            r = self.flattener.read_codes(individuals, a, b)
            self.stats["flatten_s"] += time.perf_counter() - t0
            if r is None:
                return None            # (the next lowering or load resets)
            t0 = time.perf_counter()
            codes, node_off, evals, eph_off = r
            self.ctx.lower_add(codes, node_off, evals, eph_off)
            # the population's node offsets, chunk by chunk
            np.add(np.frombuffer(node_off, dtype=np.int64)[1:], off[a - lo],
                   out=off[a - lo + 1:b - lo + 1])
            self.stats["device_s"] += time.perf_counter() - t0
            a = b
        t0 = time.perf_counter()
        depth, err, status = self.ctx.lower_end(out=self._lw_out)
        self.stats["device_s"] += time.perf_counter() - t0
        return self._lowered_batch(off, depth, err, status, keep)

    def _lowered_batch(self, off, depth, err, status, keep=True):
        """The ProgramBatch of a device lowering (None: the batch needs the
        host flattener).  *keep*: the batch outlives this call (its depth
        and error arrays are copied out of the reused output buffers)."""
        verr = None
        inexact = []
        # (the library counted the flagged trees while decoding: no scan of
        # a million zeros in the common case)
        n_err, n_status = self.ctx.lower_flags()
        if n_status:                          # rare: any flag at all
            verr = (status & 4) != 0
            if (status & 1).any():
                return None
            inexact = np.flatnonzero(status & 2).tolist()
        if n_err and ((err == ERR_CONST) & (True if verr is None else ~verr)).any():
            return None
        batch = ProgramBatch(None, off, depth.copy() if keep else depth, None,
                             err.copy() if keep else err,
                             {} if verr is None else
                             {int(i): ValueError("math domain error")
                              for i in np.flatnonzero(verr)},
                             inexact)
        batch.node_offsets = off
        batch.any_err = n_err > 0
        self.ctx.resident = batch
        self._warn_inexact(batch)
        self.stats["device_lowered"] += 1
        return batch

    def _warn_inexact(self, batch):
        """fp32 mode has no exact-integer pass: say so once."""
        if batch.inexact and self.precision == "fp32" and \
                not self._warned_inexact:
            self._warned_inexact = True
            warnings.warn("%d individual(s) may compute integers beyond "
                          "2**53; fp32 mode evaluates them in floating point "
                          "(fp64 mode keeps Python's exact ints)"
                          % len(batch.inexact), RuntimeWarning)

    def _load_exact(self, batch, individuals):
        """Programs that can compute Python ints beyond 2**53 (the batch's
        ``inexact`` candidates, decided exactly by the host flattener) are
        re-evaluated with Python-int semantics after each run
        (gpe_load_exact_v: on the device, and on the host where an int
        outgrows the device's 1088 bits); the pass reports the reference's
        exceptions (OverflowError for float(int) past 2**1024)."""
        if not batch.inexact:
            return 0
        if self.precision != "fp64" or \
                self.spec.mode not in (_lib.GPE_MODE_MSE, _lib.GPE_MODE_HITS_BOOL,
                                       _lib.GPE_MODE_SSE_SEQ):
            # no exact pass: an int constant past the float range is
            # converted, as the reference's mixed arithmetic would, and raises
            for i, exc in getattr(batch, "big_const", {}).items():
                if batch.err[i] == 0:
                    batch.err[i] = ERR_CONST
                    batch.const_exc[i] = exc
                    batch.any_err = True
            return 0
        cand = [i for i in batch.inexact if batch.err[i] == 0]
        if not cand:
            return 0
        fl = self.flattener
        if getattr(fl, "trig_leaves", None):
            # the exact pass takes sin/cos from glibc, not the leaf columns
            if self._exact_flattener is None:
                self._exact_flattener = Flattener(self.pset, self.spec.machine)
            fl = self._exact_flattener
        idx, code, off, depth, ints, _ = fl.exact_programs(
            [individuals[i] for i in cand])
        if idx:
            # kept on the batch: a reload of its programs (gpe_load_programs
            # clears the exact pass) loads the pass again (_make_resident)
            batch.exact_pass = ([cand[j] for j in idx], code, off, depth, ints)
            self.ctx.load_exact(*batch.exact_pass)
        self.stats["exact_programs"] = self.stats.get("exact_programs", 0) + len(idx)
        return len(idx)

    def prepare(self, batch, individuals):
        """Load *batch* (the programs of *individuals*) into the context and
        set up its exact-integer pass; run_batch then evaluates it."""
        self._make_resident(batch)
        if getattr(batch, "exact_pass", None) is None:
            self._load_exact(batch, individuals)

    def _make_resident(self, batch):
        # (the context tracks which batch it holds by identity: a flag on the
        # batch would not say which context, or whether another batch
        # replaced it since)
        if self.ctx.resident is batch:
            return
        if batch.code is None:
            raise RuntimeError("this device-lowered batch is no longer the "
                               "context's programs; lower or flatten it again")
        self.ctx.load_programs(batch)
        if getattr(batch, "exact_pass", None) is not None:
            self.ctx.load_exact(*batch.exact_pass)

    def run_batch(self, batch, reuse=False, want=None, out=None):
        """Device evaluation of a flattened batch → raw arrays (and the
        per-case matrix for per-case specs, else None).  *reuse*: write into
        the evaluator's kept output arrays (valid until its next call);
        *want*: the outputs to copy back (the others are None); *out*: the
        arrays to write into instead (``views(n)``, as ResultBuffers)."""
        t0 = time.perf_counter()
        self._make_resident(batch)
        cases = None
        if getattr(self.spec, "per_case", False):
            cases, hi, lo, err, flags = self.ctx.run_cases(
                self.spec.mode, self.spec.n_cases)
        else:
            hi, lo, err, flags = self.ctx.run(
                self.spec.mode, out=out if out is not None else
                self._run_out if reuse else None, want=want)
        self.stats["device_s"] += time.perf_counter() - t0
        self.stats["kernel_ms"] += self.ctx.timing()["total_ms"]
        return hi, lo, err, flags, cases

    def _want(self, batch):
        """The outputs finish_all reads (B-machine hits: the counts alone, a
        quarter of the copy at pop 1M; no error words where no program can
        raise), or None (all)."""
        want = getattr(self.spec, "outputs", None) \
            if hasattr(self.spec, "finish_all") else None
        if want is not None and getattr(batch, "exact_pass", None) is None \
                and not getattr(getattr(self.flattener, "spec", None), "has_trig", True):
            want = getattr(self.spec, "outputs_plain", want)
        return want

    def evaluate(self, individuals):
        """Fitness tuple, or the exception instance the reference would raise,
        for every individual (in order)."""
        batch = self.lower_on_device(individuals, keep=False) \
            if self.device_lowering else None
        if batch is None:
            batch = self.flatten(individuals)
        self.prepare(batch, individuals)
        want = self._want(batch)
        hi, lo, err, flags, cases = self.run_batch(batch, reuse=True, want=want)
        self.stats["calls"] += 1
        self.stats["individuals"] += len(individuals)
        self.stats["node_evals"] += batch.n_nodes() * \
            self.spec.n_cases
        if cases is None and hasattr(self.spec, "finish_all"):
            out = self.spec.finish_all(*[None if x is None else np.asarray(x)
                                         for x in (hi, lo, err, flags)])
            if getattr(batch, "any_err", True):
                for i in np.flatnonzero(batch.err).tolist():
                    out[i] = SyntaxError("too many nested parentheses") \
                        if batch.err[i] == ERR_SYNTAX else batch.const_exc[i]
            return out
        out = []
        for i in range(len(individuals)):
            code = batch.err[i]
            if code == ERR_SYNTAX:
                out.append(SyntaxError("too many nested parentheses"))
            elif code == ERR_CONST:
                out.append(batch.const_exc[i])
            elif cases is not None:
                out.append(self.spec.finish(i, hi[i], lo[i], err[i],
                                            flags[i], cases[i]))
            else:
                out.append(self.spec.finish(i, hi[i], lo[i], err[i],
                                            flags[i]))
        return out

    def map(self, individuals):
        return _yield_until_error(self.evaluate(list(individuals)))


def _yield_until_error(results):
    for res in results:
        if isinstance(res, BaseException):
            raise res
        yield res


def _unwrap(func):
    while isinstance(func, partial):
        if func.args or func.keywords:
            return None
        func = func.func
    return func if isinstance(func, GPUEvaluator) else None


def gpu_map(func, *iterables):
    """Drop-in for ``toolbox.map`` (reference default: builtin ``map``,
    ``deap/base.py:50``)."""
    ev = _unwrap(func)
    if ev is None or len(iterables) != 1:
        return map(func, *iterables)
    return ev.map(iterables[0])
