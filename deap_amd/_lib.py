"""ctypes binding of ``libgpeval.so`` (C ABI declared in ``include/gpeval.h``).

The library is built in-tree by ``__graft_entry__.build()`` /
``python -m deap_amd.build``.  There is no fallback: if the shared object is
missing or fails to load, every evaluator entry point raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DEAP_AMD_LIB: an alternative build of the same library (A/B runs)
LIB_PATH = os.environ.get("DEAP_AMD_LIB") or os.path.join(_HERE, "libgpeval.so")

GPE_MACHINE_F = 0
GPE_MACHINE_B = 1
GPE_MODE_MSE = 0
GPE_MODE_HITS_BOOL = 1
GPE_MODE_HITS_BITS = 2
GPE_MODE_SSE_NUMPY = 3
GPE_MODE_SSE_SEQ = 4
GPE_PREC_F64 = 0
GPE_PREC_F32 = 1
GPE_NO_ERROR = 0xFFFFFFFFFFFFFFFF
GPE_ERR_VALUE = 1
GPE_ERR_OVERFLOW = 2
GPE_ERR_XINT_RANGE = 3
GPE_XINT_WORDS = 34
GPE_FLAG_NONFINITE_TERM = 1
GPE_FLAG_NAN_TERM = 2
GPE_FLAG_INF_TERM = 4

# every symbol include/gpeval.h declares, with (restype, argtypes)
_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
SIGNATURES = {
    "gpe_create": (_I, [_I, ctypes.POINTER(_P)]),
    "gpe_destroy": (None, [_P]),
    "gpe_last_error": (ctypes.c_char_p, [_P]),
    "gpe_device_info": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I),
                             ctypes.c_char_p, ctypes.c_size_t]),
    "gpe_set_cases": (_I, [_P, _I, _P, _I, _I64, _P, _I]),
    "gpe_set_trig_leaves": (_I, [_P, _I]),
    "gpe_set_precision": (_I, [_P, _I]),
    "gpe_load_programs": (_I, [_P, _P, _I64, _P, _I64, _P]),
    "gpe_run": (_I, [_P, _I, _P, _P, _P, _P]),
    "gpe_run_device": (_I, [_P, _I, _P, _P, _P, _P]),
    "gpe_run_cases": (_I, [_P, _I, _P, _P, _P, _P, _P]),
    "gpe_lexicase": (_I, [_P, _P, _I64, _I64, _P, _I, ctypes.c_double, _P,
                          _I64, _P, ctypes.POINTER(_I64)]),
    "gpe_set_lowering": (_I, [_P, _I, _I, _P, _I, _P, _I]),
    "gpe_lower_programs": (_I, [_P, _P, _P, _I64, _P, _P, _P, _P, _P]),
    "gpe_lower_begin": (_I, [_P, _I64]),
    "gpe_lower_begin_into": (_I, [_P, _I64, _P, _P, _P]),
    "gpe_lower_add": (_I, [_P, _P, _P, _I64, _P, _P]),
    "gpe_lower_end": (_I, [_P, _P, _P, _P]),
    "gpe_tournament": (_I, [_P, _P, _I64, _I, ctypes.c_double, _I64, _I, _P,
                            _P]),
    "gpe_eval": (_I, [_P, _I, _P, _I64, _P, _I64, _P, _P, _P, _P, _P]),
    "gpe_last_timing": (_I, [_P, ctypes.POINTER(ctypes.c_float)]),
    "gpe_last_geometry": (_I, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "gpe_last_geometry_ex": (_I, [_P, ctypes.POINTER(ctypes.c_int64), _I]),
    "gpe_math_probe": (_I, [_P, _I, _P, _P, _I64]),
    "gpe_host_math": (_I, [_I, _P, _P, _I64]),
    "gpe_host_np_sum": (_I, [_P, _I64, _I64, _P]),
    "gpe_debug_translate": (_I, [_P, _I64, _P, _I64, _P, _I, _P, _I, _P,
                                 _I64, _P, _P]),
    "gpe_comm_unique_id": (_I, [_P]),
    "gpe_comm_init": (_I, [_P, _I, _I, _P]),
    "gpe_comm_info": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "gpe_run_sharded_device": (_I, [_P, _I, _I64, _P, _P, _P, _P]),
    "gpe_run_sharded": (_I, [_P, _I, _I64, _P, _P, _P, _P]),
    "gpe_run_gathered": (_I, [_P, _I, _I64, _P, _P, _P, _P, _P]),
    "gpe_load_exact": (_I, [_P, _P, _I64, _P, _I64, _P, _P, _P, _I64]),
    "gpe_load_exact_v": (_I, [_P, _P, _I64, _P, _I64, _P, _P, _P, _P, _I64]),
    "gpe_last_exact_host_runs": (_I, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "gpe_last_exact_host_ms": (_I, [_P, ctypes.POINTER(ctypes.c_double)]),
    "gpe_last_lower_flags": (_I, [_P, ctypes.POINTER(ctypes.c_int64),
                                  ctypes.POINTER(ctypes.c_int64)]),
    "gpe_debug_shard_combine": (_I, [_P, _I, _I64, _P, _P, _P, _P, _P, _P,
                                     _P, _P]),
    "gpe_debug_redo_union": (_I, [_P, _P, _I64]),
    "gpe_host_exact_eval": (_I, [_P, _P, _P, _I64, _P, _I, _P, _P,
                                 ctypes.POINTER(_I)]),
    "gpe_host_bigint_eval": (_I, [_P, _P, _P, _I64, _P, _I, _P, _P,
                                  ctypes.POINTER(ctypes.c_int64),
                                  ctypes.POINTER(_I)]),
    "gpe_last_comm_timing": (_I, [_P, ctypes.POINTER(ctypes.c_float)]),
    "gpe_debug_bounded_wait": (_I, [ctypes.c_double, _I64, ctypes.c_char_p,
                                    ctypes.c_size_t]),
}
GPE_E_INVALID = -1
GPE_E_COMM = -5
GPE_UNIQUE_ID_BYTES = 128

_lib = None


class GpeError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load the HIP library (raises if it is absent — no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GpeError("libgpeval.so not built (%s); run "
                       "`python -m deap_amd.build`" % path)
    # one HIP runtime per process: torch ships its own libamdhip64.so.7 and
    # whichever loads first serves both, so let torch (needed for RCCL
    # collectives in deap_amd.distributed) load it first when present
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def debug_bounded_wait(timeout_s, busy_polls):
    """The library's bounded wait on collectives, on a fake stream busy for
    *busy_polls* queries (< 0: forever): (return code, message)."""
    lib = load()
    buf = ctypes.create_string_buffer(512)
    rc = lib.gpe_debug_bounded_wait(float(timeout_s), int(busy_polls), buf,
                                    len(buf))
    return rc, buf.value.decode()


def host_math(fn, x):
    """Host-compiled twin of the kernels' sin/cos/square (CPU, no GPU)."""
    lib = load()
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.zeros_like(x)
    rc = lib.gpe_host_math(int(fn), _ptr(x), _ptr(y), len(x))
    if rc != 0:
        raise GpeError("gpe_host_math failed (%d)" % rc)
    return y


def host_np_sum(rows):
    """Host twin of the GPE_MODE_SSE_NUMPY reduction: numpy.sum of each row
    in numpy's own order (CPU, no GPU)."""
    x = np.ascontiguousarray(np.atleast_2d(rows), dtype=np.float64)
    out = np.zeros(x.shape[0])
    rc = load().gpe_host_np_sum(_ptr(x), x.shape[0], x.shape[1], _ptr(out))
    if rc != 0:
        raise GpeError("gpe_host_np_sum failed (%d)" % rc)
    return out


def debug_translate(batch, nv, table):
    """Host-only: threaded code the asm core would run (see header)."""
    lib = load()
    code = np.ascontiguousarray(batch.code, dtype=np.uint32)
    off = np.ascontiguousarray(batch.offsets, dtype=np.int64)
    depth = np.ascontiguousarray(batch.depth, dtype=np.int32)
    table = np.ascontiguousarray(table, dtype=np.uint32)
    cap = 3 * len(code) + 16
    out = np.zeros(cap, dtype=np.uint32)
    starts = np.zeros(len(depth), dtype=np.int64)
    n_out = ctypes.c_int64()
    rc = lib.gpe_debug_translate(_ptr(code), len(code), _ptr(off), len(depth),
                                 _ptr(depth), int(nv), _ptr(table),
                                 len(table), _ptr(out), cap, _ptr(starts),
                                 ctypes.byref(n_out))
    if rc != 0:
        raise GpeError("gpe_debug_translate failed (%d)" % rc)
    return out[:n_out.value], starts


def _int_rows(ints):
    """(words, off, n) of an exact pass's int table (flatten.IntTable)."""
    if ints is None or not len(ints):
        return (np.zeros(1, dtype=np.uint32), np.zeros(1, dtype=np.int64), 0)
    return (np.ascontiguousarray(ints.words, dtype=np.uint32),
            np.ascontiguousarray(ints.off, dtype=np.int64), len(ints))


def _exact_raise(rc, name):
    if rc == GPE_ERR_VALUE:
        raise ValueError("math domain error")
    if rc == GPE_ERR_OVERFLOW:
        raise OverflowError("int too large to convert to float")
    if rc == GPE_ERR_XINT_RANGE:
        from .flatten import ExactIntRangeError
        raise ExactIntRangeError("an int past the device's 1088 bits")
    if rc != 0:
        raise GpeError("%s failed (%d)" % (name, rc))


def _twos(words):
    bits = 32 * len(words)
    u = sum(int(w) << (32 * i) for i, w in enumerate(words))
    return u - (1 << bits) if bits and u >> (bits - 1) else u


def host_exact_eval(code, ints, x):
    """Host twin of the exact pass's device interpreter (test
    infrastructure, CPU): one program of Flattener.exact_programs on one
    case ``x``.  Returns the Python number the reference's evaluation gives
    (an int or a float), or raises what it raises: ValueError for sin/cos of
    an infinity, OverflowError for float(int) or int / int past the float
    range — and ExactIntRangeError where an int passes the device's 1088
    bits (the library then evaluates the program with host_bigint_eval's
    code)."""
    code = np.ascontiguousarray(code, dtype=np.uint32)
    words, off, n = _int_rows(ints)
    x = np.ascontiguousarray(np.atleast_1d(x), dtype=np.float64)
    f = ctypes.c_double()
    out = np.zeros(GPE_XINT_WORDS, dtype=np.uint32)
    isint = _I()
    rc = load().gpe_host_exact_eval(_ptr(code), _ptr(words), _ptr(off), n,
                                    _ptr(x), len(x), ctypes.byref(f),
                                    _ptr(out), ctypes.byref(isint))
    _exact_raise(rc, "gpe_host_exact_eval")
    return _twos(out.tolist()) if isint.value else f.value


def host_bigint_eval(code, ints, x):
    """The exact pass's host evaluator with unbounded ints (the one the
    library runs for programs past the device's 1088 bits), on one case:
    the Python number or the exception, as host_exact_eval."""
    code = np.ascontiguousarray(code, dtype=np.uint32)
    words, off, n = _int_rows(ints)
    x = np.ascontiguousarray(np.atleast_1d(x), dtype=np.float64)
    f = ctypes.c_double()
    isint = _I()
    cap = ctypes.c_int64(64)
    lib = load()
    while True:
        out = np.zeros(max(cap.value, 1), dtype=np.uint32)
        want = cap.value
        rc = lib.gpe_host_bigint_eval(_ptr(code), _ptr(words), _ptr(off), n,
                                      _ptr(x), len(x), ctypes.byref(f),
                                      _ptr(out), ctypes.byref(cap),
                                      ctypes.byref(isint))
        if rc == GPE_E_INVALID and cap.value > want:
            continue                          # a wider int: again, with room
        break
    _exact_raise(rc, "gpe_host_bigint_eval")
    return _twos(out[:cap.value].tolist()) if isint.value else f.value


def comm_unique_id():
    """The communicator id rank 0 creates (gpe_comm_unique_id): bytes."""
    buf = ctypes.create_string_buffer(GPE_UNIQUE_ID_BYTES)
    rc = load().gpe_comm_unique_id(buf)
    if rc != 0:
        raise GpeError("gpe_comm_unique_id failed (%d): is librccl.so.1 "
                       "available?" % rc)
    return buf.raw


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class _Buffers(object):
    """Output arrays kept across calls (grown, never shrunk): a fresh
    million-entry array per call is fresh pages, and their first-touch
    faults (and the unmapping when Python frees them) were ~3 ms of an
    ``evaluate`` at pop 1M.  The caller owns the contents only until its
    next call with the same buffers."""
    dtypes = ()

    def __init__(self):
        self._arrays = [np.zeros(0, dtype=d) for d in self.dtypes]

    def views(self, n):
        if len(self._arrays[0]) < n:
            cap = max(n, 2 * len(self._arrays[0]))
            self._arrays = [np.zeros(cap, dtype=d) for d in self.dtypes]
        return tuple(a[:n] for a in self._arrays)


class ResultBuffers(_Buffers):
    """(hi, lo, err, flags) of :meth:`Context.run`."""
    dtypes = (np.float64, np.float64, np.uint64, np.uint32)


class LoweringBuffers(_Buffers):
    """(depth, err, status) of :meth:`Context.lower_programs`."""
    dtypes = (np.int32, np.uint8, np.uint8)


class Context(object):
    """One device context (one per process/GPU)."""

    def __init__(self, device=0):
        self.lib = load()
        handle = ctypes.c_void_p()
        rc = self.lib.gpe_create(int(device), ctypes.byref(handle))
        if rc != 0:
            raise GpeError("gpe_create(%d) failed with %d" % (device, rc))
        self.h = handle
        self.device = device
        self.machine = None
        self.n_prog = 0
        # the ProgramBatch whose programs are loaded (identity; None after a
        # device lowering until its caller names the batch it built)
        self.resident = None
        # an open chunked lowering: its tree count, and the output arrays
        # gpe_lower_begin_into was given (None: outputs at lower_end)
        self._lw_n = 0
        self._lw_into = None

    def close(self):
        if getattr(self, "h", None):
            self.lib.gpe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.gpe_last_error(self.h)
            raise GpeError("%s failed (%d): %s" % (what, rc,
                                                   msg.decode() if msg else ""))

    def device_info(self):
        cu, clk = ctypes.c_int(), ctypes.c_int()
        name = ctypes.create_string_buffer(256)
        self._check(self.lib.gpe_device_info(self.h, ctypes.byref(cu),
                                             ctypes.byref(clk), name, 256),
                    "gpe_device_info")
        return {"cu": cu.value, "clock_khz": clk.value,
                "arch": name.value.decode()}

    def set_cases(self, machine, X, terms):
        X = np.ascontiguousarray(X)
        terms = None if terms is None else np.ascontiguousarray(terms)
        if machine == GPE_MACHINE_F:
            X = X.astype(np.float64, copy=False)
            n_vars, n_cases = X.shape
            if terms is not None:
                terms = terms.astype(np.float64, copy=False)
                if terms.ndim == 1:
                    terms = terms[None, :]
                assert terms.shape[1] == n_cases
            n_terms = 0 if terms is None else terms.shape[0]
        else:
            raise ValueError("use set_bitplanes for the B machine")
        self._check(self.lib.gpe_set_cases(self.h, machine, _ptr(X), n_vars,
                                           n_cases, _ptr(terms), n_terms),
                    "gpe_set_cases")
        self.machine = machine
        self._keep = (X, terms)

    def set_trig_leaves(self, enable):
        """Device columns sin(x_v), cos(x_v) per run (see gpeval.h)."""
        self._check(self.lib.gpe_set_trig_leaves(self.h, int(bool(enable))),
                    "gpe_set_trig_leaves")
        self.n_prog = 0
        self.resident = None

    def set_precision(self, prec):
        """GPE_PREC_F64 (default) or GPE_PREC_F32 for the F machine."""
        self._check(self.lib.gpe_set_precision(self.h, int(prec)),
                    "gpe_set_precision")

    def set_bitplanes(self, planes, out_plane, n_cases):
        planes = np.ascontiguousarray(planes, dtype=np.uint32)
        out_plane = np.ascontiguousarray(out_plane, dtype=np.uint32)
        self._check(self.lib.gpe_set_cases(self.h, GPE_MACHINE_B,
                                           _ptr(planes), planes.shape[0],
                                           int(n_cases), _ptr(out_plane), 1),
                    "gpe_set_cases")
        self.machine = GPE_MACHINE_B
        self._keep = (planes, out_plane)

    def load_programs(self, batch):
        code = np.ascontiguousarray(batch.code, dtype=np.uint32)
        off = np.ascontiguousarray(batch.offsets, dtype=np.int64)
        depth = np.ascontiguousarray(batch.depth, dtype=np.int32)
        self._check(self.lib.gpe_load_programs(self.h, _ptr(code), len(code),
                                               _ptr(off), len(depth),
                                               _ptr(depth)),
                    "gpe_load_programs")
        self.n_prog = len(depth)
        self.resident = batch

    def load_exact(self, progs, code, offsets, depth, ints):
        """gpe_load_exact_v: re-evaluate the loaded programs ``progs`` with
        Python-int semantics after every run (Flattener.exact_programs)."""
        progs = np.ascontiguousarray(progs, dtype=np.int32)
        code = np.ascontiguousarray(code, dtype=np.uint32)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        depth = np.ascontiguousarray(depth, dtype=np.int32)
        words, woff, n = _int_rows(ints)
        self._check(self.lib.gpe_load_exact_v(
            self.h, _ptr(progs), len(progs), _ptr(code), len(code), _ptr(off),
            _ptr(depth), _ptr(words), _ptr(woff), n), "gpe_load_exact_v")

    def lower_flags(self):
        """(trees with a nonzero error code, with a nonzero status) of the
        last device lowering (gpe_last_lower_flags)."""
        ne, ns = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.gpe_last_lower_flags(self.h, ctypes.byref(ne), ctypes.byref(ns)),
                    "gpe_last_lower_flags")
        return ne.value, ns.value

    def exact_host_runs(self):
        """Exact-pass programs the last run evaluated on the host (ints past
        the device's 1088 bits)."""
        n = ctypes.c_int64()
        self._check(self.lib.gpe_last_exact_host_runs(self.h, ctypes.byref(n)),
                    "gpe_last_exact_host_runs")
        return n.value

    def exact_host_ms(self):
        """Wall time of the last run's host exact pass, ms."""
        ms = ctypes.c_double()
        self._check(self.lib.gpe_last_exact_host_ms(self.h, ctypes.byref(ms)),
                    "gpe_last_exact_host_ms")
        return ms.value

    def debug_shard_combine(self, parts, errs, flags, case_offsets):
        """gpe_debug_shard_combine (test infrastructure): the case-sharded
        combine of ``world`` ranks' outputs on this device.  parts
        [world, 2, n] float64, errs [world, n] uint64, flags [world, n]
        uint32, case_offsets [world]; returns (hi, lo, err, flags)."""
        parts = np.ascontiguousarray(parts, dtype=np.float64)
        errs = np.ascontiguousarray(errs, dtype=np.uint64)
        flags = np.ascontiguousarray(flags, dtype=np.uint32)
        offs = np.ascontiguousarray(case_offsets, dtype=np.int64)
        world, _, n = parts.shape
        hi, lo = np.zeros(n), np.zeros(n)
        err = np.zeros(n, dtype=np.uint64)
        fl = np.zeros(n, dtype=np.uint32)
        self._check(self.lib.gpe_debug_shard_combine(
            self.h, world, n, _ptr(parts), _ptr(errs), _ptr(flags), _ptr(offs),
            _ptr(hi), _ptr(lo), _ptr(err), _ptr(fl)), "gpe_debug_shard_combine")
        return hi, lo, err, fl

    def debug_redo_union(self, flags):
        """gpe_debug_redo_union (test infrastructure): redo flags other
        ranks raised, ORed into every later run's own (None clears)."""
        f = np.zeros(0, dtype=np.uint32) if flags is None else \
            np.ascontiguousarray(flags, dtype=np.uint32)
        self._check(self.lib.gpe_debug_redo_union(self.h, _ptr(f) if len(f) else None,
                                                  len(f)), "gpe_debug_redo_union")

    def run(self, mode, out=None, want=None):
        """gpe_run → (hi, lo, err, flags).  *out*: a :class:`ResultBuffers`
        to write into (views of its arrays are returned), else fresh arrays.
        *want*: the names of the outputs to copy back (default all); the
        others are returned as None (gpe_run's NULL outputs)."""
        n = self.n_prog
        if out is not None:
            arrs = list(out.views(n))
        else:
            arrs = [np.zeros(n, dtype=np.float64), np.zeros(n, dtype=np.float64),
                    np.zeros(n, dtype=np.uint64), np.zeros(n, dtype=np.uint32)]
        if want is not None:
            arrs = [a if name in want else None
                    for a, name in zip(arrs, ("hi", "lo", "err", "flags"))]
        if n:
            self._check(self.lib.gpe_run(self.h, mode, *[
                _ptr(a) if a is not None else None for a in arrs]), "gpe_run")
        return tuple(arrs)

    def run_cases(self, mode, n_cases):
        """gpe_run plus the per-case terms ``[n_prog, n_cases]``."""
        n = self.n_prog
        cases = np.zeros((n, n_cases), dtype=np.float64)
        hi = np.zeros(n, dtype=np.float64)
        lo = np.zeros(n, dtype=np.float64)
        err = np.zeros(n, dtype=np.uint64)
        flags = np.zeros(n, dtype=np.uint32)
        if n:
            self._check(self.lib.gpe_run_cases(self.h, mode, _ptr(cases),
                                               _ptr(hi), _ptr(lo), _ptr(err),
                                               _ptr(flags)), "gpe_run_cases")
        return cases, hi, lo, err, flags

    def lexicase(self, values, maximise, k, rng, mode=0, epsilon=0.0):
        """gpe_lexicase: k selections on ``values`` [n, n_cases] (None: the
        last run_cases matrix), drawing from the ``random.Random``-compatible
        ``rng`` exactly as the reference does and advancing its state.
        Returns (indices, failed): failed is -1 or the selection at which no
        candidate was left (the reference's IndexError)."""
        version, words, gauss = rng.getstate()
        st = np.asarray(words, dtype=np.uint32)
        maximise = np.ascontiguousarray(maximise, dtype=np.uint8)
        if values is None:
            n, c, ptr = 0, len(maximise), None
        else:
            values = np.ascontiguousarray(values, dtype=np.float64)
            n, c = values.shape
            ptr = _ptr(values)
        out = np.zeros(max(int(k), 1), dtype=np.int32)
        failed = ctypes.c_int64(-1)
        self._check(self.lib.gpe_lexicase(self.h, ptr, n, c, _ptr(maximise),
                                          int(mode), float(epsilon),
                                          _ptr(st), int(k), _ptr(out),
                                          ctypes.byref(failed)),
                    "gpe_lexicase")
        rng.setstate((version, tuple(int(w) for w in st), gauss))
        done = int(k) if failed.value < 0 else failed.value
        return out[:done], failed.value

    def set_lowering(self, machine, nv, leaf, entries, n_entries):
        """gpe_set_lowering: the pset tables of device lowering (``leaf``
        one byte per argument, ``entries`` packed gpe_entry records)."""
        leaf = bytes(leaf)
        self._lw = (leaf, bytes(entries))        # keep the buffers alive
        lb = ctypes.create_string_buffer(leaf, max(len(leaf), 1))
        eb = ctypes.create_string_buffer(self._lw[1], max(len(self._lw[1]), 1))
        self._check(self.lib.gpe_set_lowering(self.h, int(machine), int(nv), lb,
                                              len(leaf), eb, int(n_entries)),
                    "gpe_set_lowering")

    def lower_programs(self, codes, node_off, evals, eph_off, out=None):
        """gpe_lower_programs: lower the trees on the device and load them.
        Returns (depth int32[n], err uint8[n], status uint8[n]) — views of
        *out*'s (a :class:`LoweringBuffers`) arrays when given."""
        node_off = np.frombuffer(node_off, dtype=np.int64)
        eph_off = np.frombuffer(eph_off, dtype=np.int64)
        n = len(node_off) - 1
        if out is not None:
            depth, err, status = out.views(max(n, 1))
        else:
            depth = np.zeros(max(n, 1), dtype=np.int32)
            err = np.zeros(max(n, 1), dtype=np.uint8)
            status = np.zeros(max(n, 1), dtype=np.uint8)
        cb = np.frombuffer(codes, dtype=np.uint8) if len(codes) else \
            np.zeros(1, dtype=np.uint8)
        eb = np.frombuffer(evals, dtype=np.uint8) if len(evals) else \
            np.zeros(1, dtype=np.uint8)
        self.resident = None
        self.n_prog = 0
        self._check(self.lib.gpe_lower_programs(
            self.h, _ptr(cb), _ptr(node_off), n, _ptr(eb), _ptr(eph_off),
            _ptr(depth), _ptr(err), _ptr(status)), "gpe_lower_programs")
        self.n_prog = n
        return depth[:n], err[:n], status[:n]

    def lower_begin(self, n_total, out=None):
        """gpe_lower_begin: a device lowering of n_total trees, added in
        chunks (:meth:`lower_add`) and finished by :meth:`lower_end`.  With
        *out* (a :class:`LoweringBuffers`), gpe_lower_begin_into: the chunks
        are decoded into *out*'s arrays as they are added, and lower_end
        returns views of them."""
        self.resident = None
        self.n_prog = 0
        self._lw_n = int(n_total)
        self._lw_into = None
        if out is not None and n_total > 0:
            depth, err, status = out.views(int(n_total))
            self._check(self.lib.gpe_lower_begin_into(
                self.h, int(n_total), _ptr(depth), _ptr(err), _ptr(status)),
                "gpe_lower_begin_into")
            self._lw_into = (depth, err, status)
            return
        self._check(self.lib.gpe_lower_begin(self.h, int(n_total)), "gpe_lower_begin")

    def lower_add(self, codes, node_off, evals, eph_off):
        """gpe_lower_add: the next chunk (read_codes' four buffers, offsets
        from 0); its upload and lowering run on the device asynchronously."""
        node_off = np.frombuffer(node_off, dtype=np.int64)
        eph_off = np.frombuffer(eph_off, dtype=np.int64)
        n = len(node_off) - 1
        cb = np.frombuffer(codes, dtype=np.uint8) if len(codes) else \
            np.zeros(1, dtype=np.uint8)
        eb = np.frombuffer(evals, dtype=np.uint8) if len(evals) else \
            np.zeros(1, dtype=np.uint8)
        self._check(self.lib.gpe_lower_add(self.h, _ptr(cb), _ptr(node_off), n,
                                           _ptr(eb), _ptr(eph_off)), "gpe_lower_add")

    def lower_add_addr(self):
        """The address of gpe_lower_add (for the native read-and-lower
        pipeline, Flattener.read_lower)."""
        return ctypes.cast(self.lib.gpe_lower_add, ctypes.c_void_p).value

    def handle_addr(self):
        return ctypes.cast(self.h, ctypes.c_void_p).value

    def check_rc(self, rc, what):
        self._check(int(rc), what)

    def lower_end(self, out=None):
        """gpe_lower_end → (depth int32[n], err uint8[n], status uint8[n])
        for all the lowering's trees (views of *out*'s arrays when given)."""
        n = self._lw_n
        into, self._lw_into = self._lw_into, None
        if into is not None:
            depth, err, status = into
        elif out is not None:
            depth, err, status = out.views(max(n, 1))
        else:
            depth = np.zeros(max(n, 1), dtype=np.int32)
            err = np.zeros(max(n, 1), dtype=np.uint8)
            status = np.zeros(max(n, 1), dtype=np.uint8)
        self._check(self.lib.gpe_lower_end(self.h, _ptr(depth), _ptr(err), _ptr(status)),
                    "gpe_lower_end")
        self.n_prog = n
        self.resident = None
        return depth[:n], err[:n], status[:n]

    def tournament(self, wvalues, k, tournsize, rng, weight=1.0):
        """gpe_tournament: k tournaments of ``tournsize`` on ``wvalues``
        [n] or [n, nobj] (None: the last run's fitness on the device times
        ``weight``), drawing from the ``random.Random``-compatible ``rng`` as
        the reference's selTournament does and advancing its state.
        Returns the selected indices."""
        version, words, gauss = rng.getstate()
        st = np.asarray(words, dtype=np.uint32)
        if wvalues is None:
            n, nobj, ptr = 0, 1, None
        else:
            wvalues = np.ascontiguousarray(wvalues, dtype=np.float64)
            if wvalues.ndim == 1:
                wvalues = wvalues[:, None]
            n, nobj = wvalues.shape
            ptr = _ptr(wvalues)
        out = np.zeros(max(int(k), 1), dtype=np.int32)
        self._check(self.lib.gpe_tournament(self.h, ptr, n, nobj, float(weight),
                                            int(k), int(tournsize), _ptr(st),
                                            _ptr(out)), "gpe_tournament")
        rng.setstate((version, tuple(int(w) for w in st), gauss))
        return out[:int(k)]

    def run_device(self, mode, hi_ptr, lo_ptr, err_ptr, flags_ptr):
        self._check(self.lib.gpe_run_device(self.h, mode, hi_ptr, lo_ptr,
                                            err_ptr, flags_ptr),
                    "gpe_run_device")

    # ---- multi-GPU (include/gpeval.h: gpe_comm_*, gpe_run_sharded*) ----
    def comm_init(self, rank, world, unique_id):
        """Join the RCCL communicator ``unique_id`` (from rank 0's
        :func:`comm_unique_id`) as ``rank`` of ``world``.  Collective."""
        uid = ctypes.create_string_buffer(bytes(unique_id),
                                          GPE_UNIQUE_ID_BYTES)
        self._check(self.lib.gpe_comm_init(self.h, int(rank), int(world),
                                           uid), "gpe_comm_init")

    def comm_info(self):
        r, w = _I(), _I()
        self._check(self.lib.gpe_comm_info(self.h, ctypes.byref(r),
                                           ctypes.byref(w)), "gpe_comm_info")
        return r.value, w.value

    def run_sharded(self, mode, case_offset):
        """Case-sharded gpe_run: whole-population (hi, lo, err, flags),
        identical on every rank.  Collective."""
        n = self.n_prog
        hi = np.zeros(n, dtype=np.float64)
        lo = np.zeros(n, dtype=np.float64)
        err = np.zeros(n, dtype=np.uint64)
        flags = np.zeros(n, dtype=np.uint32)
        self._check(self.lib.gpe_run_sharded(self.h, mode, int(case_offset),
                                             _ptr(hi), _ptr(lo), _ptr(err),
                                             _ptr(flags)), "gpe_run_sharded")
        return hi, lo, err, flags

    def run_sharded_device(self, mode, case_offset, hi_ptr=None, lo_ptr=None,
                           err_ptr=None, flags_ptr=None):
        self._check(self.lib.gpe_run_sharded_device(
            self.h, mode, int(case_offset), hi_ptr, lo_ptr, err_ptr,
            flags_ptr), "gpe_run_sharded_device")

    def run_gathered(self, mode, width, world, tags=None, want=None):
        """Population-sharded gpe_run: every rank's results, rank r's
        program i at r * width + i; ``tags`` (uint8 per loaded program)
        come back in bits 8..15 of the flags.  *want*: the outputs to copy
        (default all; the others are None — the flags always come, they
        carry the tags).  Collective."""
        m = int(width) * int(world)
        if tags is not None:
            tags = np.ascontiguousarray(tags, dtype=np.uint8)
        names = ("hi", "lo", "err", "flags")
        dts = (np.float64, np.float64, np.uint64, np.uint32)
        arrs = [np.zeros(m, dtype=d) if (want is None or nm in want or
                                         nm == "flags") else None
                for nm, d in zip(names, dts)]
        self._check(self.lib.gpe_run_gathered(self.h, mode, int(width),
                                              _ptr(tags), *[
                                                  _ptr(a) if a is not None else None
                                                  for a in arrs]),
                    "gpe_run_gathered")
        return tuple(arrs)

    def timing(self):
        ms = (ctypes.c_float * 3)()
        self._check(self.lib.gpe_last_timing(self.h, ms), "gpe_last_timing")
        return {"kernel_ms": ms[0], "reduce_ms": ms[1], "total_ms": ms[2]}

    def comm_timing(self):
        """Collective time of the last sharded / gathered run (waits for it,
        bounded by GPE_COMM_TIMEOUT_S)."""
        ms = (ctypes.c_float * 2)()
        self._check(self.lib.gpe_last_comm_timing(self.h, ms),
                    "gpe_last_comm_timing")
        return {"comm_ms": ms[0], "redo_ms": ms[1]}

    def math_probe(self, fn, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros_like(x)
        self._check(self.lib.gpe_math_probe(self.h, int(fn), _ptr(x), _ptr(y),
                                            len(x)), "gpe_math_probe")
        return y

    def geometry(self):
        g = (ctypes.c_int64 * 17)()
        self._check(self.lib.gpe_last_geometry_ex(self.h, g, 17),
                    "gpe_last_geometry_ex")
        return dict(zip(("asm", "fast", "deep", "redo", "P", "groups",
                         "redo_tiles", "waves_per_block", "asm_deep",
                         "asm_deep_P", "asm_deep_groups",
                         "asm_deep_waves_per_block", "redo_exact_cpp",
                         "asm_typed", "asm_typed_P", "asm_typed_groups",
                         "typed_const"),
                        list(g)))
