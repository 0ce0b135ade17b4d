"""Multi-GPU evaluation over one node: one process per GPU.

The reference has no distributed evaluation of its own; its only parallelism
is a user-registered ``multiprocessing.Pool.map`` over individuals
(``examples/ga/onemax_mp.py:58-59``, ``doc/tutorials/basic/part4.rst:19-56``).
Two MI355X-native decompositions replace it:

* :class:`PopulationSharded` — individuals are split into contiguous ranges of
  equal total tree length; each rank evaluates its range on the full (small)
  case set; results are all-gathered.  Bit-identical to one GPU.  (config 3)
* :class:`CaseSharded` — every rank holds a contiguous slice of the fitness
  cases and evaluates every individual on it; the per-individual partial SSE
  (double-double hi/lo) is all-gathered and summed in rank order, the
  first-error case index reduced with MIN and the flag bits OR-ed.
  (config 4)

The collectives run in the C ABI when the local evaluator owns a device
context: ``libgpeval.so`` holds an RCCL communicator (``gpe_comm_init``;
``gpe_run_sharded`` / ``gpe_run_gathered`` reduce on the context's stream,
no host round trip).  torch.distributed serves only to hand rank 0's
communicator id to the other ranks (through its key-value store) and, for
CPU stand-ins of the device (the gloo tests), as the host fallback that
performs the same reductions in the same order.

Both wrap a *local* evaluator exposing ``flatten(individuals)``,
``run_batch(batch) -> (hi, lo, err, flags, cases)``, ``spec`` and, for the
native path, ``ctx`` — normally a :class:`deap_amd.evaluator.GPUEvaluator`
bound to this rank's GPU (``LOCAL_RANK``).
"""
import itertools

import numpy as np

from . import _lib
from .flatten import ERR_CONST, ERR_SYNTAX

__all__ = ["shard_range", "balanced_ranges", "PopulationSharded",
           "CaseSharded"]

_I64_NONE = np.iinfo(np.int64).max
_FLAG_BITS = 3              # GPE_FLAG_NONFINITE_TERM | NAN_TERM | INF_TERM


def shard_range(n, rank, world):
    """Contiguous [lo, hi) share of n items for *rank*."""
    return rank * n // world, (rank + 1) * n // world


def balanced_ranges(lengths, world):
    """Split indices 0..n into *world* contiguous ranges of ~equal total
    length (the interpreter's work is linear in tree length)."""
    lengths = np.asarray(lengths, dtype=np.int64)
    csum = np.concatenate([[0], np.cumsum(lengths)])
    total = csum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(csum, total * r / world,
                                        side="left")))
    cuts.append(len(lengths))
    cuts = np.maximum.accumulate(np.asarray(cuts))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def _lengths(individuals):
    """len() of every individual (tree lists read by native threads)."""
    try:
        from . import _flatnative
        b = _flatnative.lengths(individuals)
    except ImportError:
        b = None
    if b is not None:
        return np.frombuffer(b, dtype=np.int64)
    return np.fromiter(map(len, individuals), dtype=np.int64,
                       count=len(individuals))


def _torch_dist(local=None):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        raise RuntimeError("torch.distributed is not initialised")
    dev = torch.device("cpu")
    if dist.get_backend() == "nccl":
        # the local evaluator's device, not torch's current one
        ctx = getattr(local, "ctx", None)
        dev = torch.device("cuda", ctx.device if ctx is not None
                           else torch.cuda.current_device())
    return torch, dist, dev


_COMM_SEQ = itertools.count()


def native_comm(local):
    """The local evaluator's context with its RCCL communicator joined, or
    None for the host fallback (no device context, or a gloo process
    group: CPU stand-ins, or several ranks sharing one GPU, which RCCL does
    not allow).  The communicator id travels through torch.distributed's
    key-value store — no collective, no device buffer."""
    ctx = getattr(local, "ctx", None)
    if ctx is None:
        return None
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_backend() != "nccl":
        return None
    rank, world = dist.get_rank(), dist.get_world_size()
    if ctx.comm_info() == (rank, world):
        return ctx
    store = dist.distributed_c10d._get_default_store()
    key = "deap_amd/comm/%d" % next(_COMM_SEQ)
    if rank == 0:
        store.set(key, _lib.comm_unique_id())
    uid = store.get(key)
    ctx.comm_init(rank, world, uid)
    return ctx


def _check_shardable(spec, case_sharded):
    if getattr(spec, "per_case", False):
        raise NotImplementedError("per-case outputs are not gathered across "
                                  "ranks; evaluate per-case specs on one GPU")
    if case_sharded and spec.mode in (_lib.GPE_MODE_SSE_NUMPY,
                                      _lib.GPE_MODE_SSE_SEQ):
        raise NotImplementedError("numpy.sum / builtin sum orders are "
                                  "single-device reductions; use "
                                  "PopulationSharded for these specs")


def _prepare(local, batch, individuals):
    """The local evaluator's prepare (program load + exact-integer pass);
    stand-ins without one load nothing here."""
    prep = getattr(local, "prepare", None)
    if prep is not None:
        prep(batch, individuals)


def _rebuilt_exc(local, individual, code):
    """The exception of a flattener verdict another rank made."""
    return local.flatten([individual]).const_exc[0]


def _finish(spec, batch, hi, lo, err, flags):
    out = []
    for i in range(len(batch)):
        code = batch.err[i]
        if code == ERR_SYNTAX:
            out.append(SyntaxError("too many nested parentheses"))
        elif code == ERR_CONST:
            out.append(batch.const_exc[i])
        else:
            out.append(spec.finish(i, hi[i], lo[i], err[i], flags[i]))
    return out


class PopulationSharded(object):
    """Each rank evaluates a length-balanced contiguous slice of the
    population; results are all-gathered (no reduction: bit-identical)."""

    def __init__(self, local):
        self.local = local
        self.spec = local.spec

    def evaluate(self, individuals):
        _check_shardable(self.spec, False)
        torch, dist, dev = _torch_dist(self.local)
        rank, world = dist.get_rank(), dist.get_world_size()
        if not isinstance(individuals, list):
            individuals = list(individuals)
        ranges = balanced_ranges(_lengths(individuals), world)
        lo_i, hi_i = ranges[rank]
        width = max(max(b - a for a, b in ranges), 1)
        # (the whole list when this rank holds it all: a 1M-entry slice
        # and its release are ~5 ms of pure overhead)
        mine = individuals if (lo_i, hi_i) == (0, len(individuals)) else \
            individuals[lo_i:hi_i]
        ctx = native_comm(self.local)
        batch = None
        if ctx is not None and getattr(self.local, "device_lowering", False) \
                and mine:
            batch = self.local.lower_on_device(mine)   # loads the programs
        if batch is None:
            batch = self.local.flatten(mine)
        _prepare(self.local, batch, mine)
        if ctx is not None:
            return self._evaluate_native(ctx, individuals, ranges, width,
                                         batch)
        n = len(batch)
        vals = torch.zeros(4, width, dtype=torch.float64, device=dev)
        errs = torch.full((width,), -1, dtype=torch.int64, device=dev)
        if n:
            h, l, e, f = self.local.run_batch(batch)[:4]
            vals[0, :n] = torch.from_numpy(np.asarray(h, np.float64)).to(dev)
            vals[1, :n] = torch.from_numpy(np.asarray(l, np.float64)).to(dev)
            vals[2, :n] = torch.from_numpy(np.asarray(f, np.float64)).to(dev)
            vals[3, :n] = torch.from_numpy(
                batch.err.astype(np.float64)).to(dev)
            errs[:n] = torch.from_numpy(
                np.asarray(e, np.uint64).view(np.int64).copy()).to(dev)
        gv = [torch.empty_like(vals) for _ in range(world)]
        ge = [torch.empty_like(errs) for _ in range(world)]
        dist.all_gather(gv, vals)
        dist.all_gather(ge, errs)
        out = []
        for r, (a, b) in enumerate(ranges):
            v = gv[r].cpu().numpy()
            e = ge[r].cpu().numpy().view(np.uint64)
            for k in range(b - a):
                code = int(v[3, k])
                if code == ERR_SYNTAX:
                    out.append(SyntaxError("too many nested parentheses"))
                elif code == ERR_CONST:  # rare: rebuild it
                    out.append(_rebuilt_exc(self.local, individuals[a + k],
                                            code))
                else:
                    out.append(self.spec.finish(a + k, v[0, k], v[1, k],
                                                e[k], int(v[2, k])))
        return out

    def _evaluate_native(self, ctx, individuals, ranges, width, batch):
        """gpe_run_gathered: this rank's slice on its GPU, every rank's
        (hi, lo, err, flags) all-gathered over RCCL; the flattener's
        per-tree verdicts (SyntaxError, constant-subtree exception) travel
        as tags in the flag word."""
        fa = hasattr(self.spec, "finish_all")
        want = getattr(self.spec, "outputs", None) if fa else None
        hi, lo, err, flags = ctx.run_gathered(
            self.spec.mode, width, len(ranges),
            np.asarray(batch.err, dtype=np.uint8), want=want)
        # the gathered slots of real programs, in population order (already
        # so when no rank's slice is shorter than the width)
        if any(b - a != width for a, b in ranges):
            idx = np.concatenate([r * width + np.arange(b - a, dtype=np.int64)
                                  for r, (a, b) in enumerate(ranges)])
            hi, lo, err, flags = [None if x is None else x[idx]
                                  for x in (hi, lo, err, flags)]
        tags = flags >> 8
        flags = flags & np.uint32(0xff)
        if fa:
            out = self.spec.finish_all(hi, lo, err, flags)
        else:
            n = sum(b - a for a, b in ranges)
            out = [self.spec.finish(i, hi[i], lo[i], err[i], int(flags[i]))
                   for i in range(n)]
        for i in np.flatnonzero(tags).tolist():
            tag = int(tags[i])
            if tag == ERR_SYNTAX:
                out[i] = SyntaxError("too many nested parentheses")
            elif tag == ERR_CONST:       # rare: rebuild it
                out[i] = _rebuilt_exc(self.local, individuals[i], tag)
        return out

    def map(self, individuals):
        from .evaluator import _yield_until_error
        return _yield_until_error(self.evaluate(individuals))


class CaseSharded(object):
    """Each rank owns cases [lo, hi); partial SSEs are all-reduced.

    *local* must already hold this rank's case slice; *n_total* is the total
    case count (the MSE denominator) and *case_offset* this rank's first
    case (to report the global index of the first failing case).
    With a device context the reduction is ``gpe_run_sharded`` (RCCL in
    the C ABI: the (hi, lo) partials all-gathered and summed as
    double-doubles in rank order).  The host fallback (gloo, CPU stand-ins)
    does the same with ``reduce="allgather"`` (the default), or sums hi and
    lo separately with one all-reduce (``reduce="allreduce"``: fewer bytes,
    rank-order dependent in the last bits)."""

    def __init__(self, local, n_total, case_offset, reduce="allgather"):
        self.local = local
        self.spec = local.spec
        self.n_total = n_total
        self.case_offset = case_offset
        self.reduce = reduce

    def evaluate(self, individuals):
        _check_shardable(self.spec, True)
        torch, dist, dev = _torch_dist(self.local)
        individuals = list(individuals)
        batch = self.local.flatten(individuals)
        n = len(batch)
        if n == 0:
            return []
        _prepare(self.local, batch, individuals)
        ctx = native_comm(self.local)
        if ctx is not None:
            hi, lo, err, flags = ctx.run_sharded(self.spec.mode,
                                                 self.case_offset)
            return self._finish(batch, hi, lo, err, flags)
        h, l, e, f = self.local.run_batch(batch)[:4]
        e = np.asarray(e, dtype=np.uint64)
        none = e == np.uint64(_lib.GPE_NO_ERROR)
        eg = np.where(none, _I64_NONE,
                      (e + (np.uint64(self.case_offset) << np.uint64(2)))
                      .astype(np.int64))
        err_t = torch.from_numpy(eg).to(dev)
        # flags are bit sets: OR over ranks = MAX of each bit (RCCL has no
        # bitwise reduction)
        bits = (np.asarray(f, dtype=np.int64)[None, :] >>
                np.arange(_FLAG_BITS, dtype=np.int64)[:, None]) & 1
        flag_t = torch.from_numpy(np.ascontiguousarray(bits)).to(dev)
        dist.all_reduce(err_t, op=dist.ReduceOp.MIN)
        dist.all_reduce(flag_t, op=dist.ReduceOp.MAX)
        if self.reduce == "allgather":
            mine = torch.from_numpy(np.stack([h, l]).astype(np.float64)).to(
                dev)
            parts = [torch.empty_like(mine)
                     for _ in range(dist.get_world_size())]
            dist.all_gather(parts, mine)
            hs = [p.cpu().numpy() for p in parts]
            hi, lo = _dd_sum_ranks(hs)
        else:
            both = torch.from_numpy(np.stack([h, l]).astype(np.float64)).to(
                dev)
            dist.all_reduce(both, op=dist.ReduceOp.SUM)
            hi, lo = both.cpu().numpy()
        eg = err_t.cpu().numpy()
        err = np.where(eg == _I64_NONE, np.uint64(_lib.GPE_NO_ERROR),
                       eg.astype(np.uint64))
        flags = (flag_t.cpu().numpy() << np.arange(
            _FLAG_BITS, dtype=np.int64)[:, None]).sum(axis=0).astype(np.uint32)
        return self._finish(batch, hi, lo, err, flags)

    def _finish(self, batch, hi, lo, err, flags):
        saved = self.spec.n_cases
        self.spec.n_cases = self.n_total
        try:
            return _finish(self.spec, batch, hi, lo, err, flags)
        finally:
            self.spec.n_cases = saved

    def map(self, individuals):
        from .evaluator import _yield_until_error
        return _yield_until_error(self.evaluate(individuals))


def _two_sum(a, b):
    s = a + b
    bb = s - a
    e = (a - (s - bb)) + (b - bb)
    return s, np.where(np.isfinite(s), e, 0.0)


def _dd_sum_ranks(parts):
    hi = np.zeros_like(parts[0][0])
    lo = np.zeros_like(parts[0][0])
    with np.errstate(invalid="ignore", over="ignore"):
        for p in parts:
            s, e = _two_sum(hi, p[0])
            e = e + (lo + p[1])
            h = s + e
            lo = np.where(np.isfinite(h), e - (h - s), 0.0)
            hi = h
    return hi, lo
