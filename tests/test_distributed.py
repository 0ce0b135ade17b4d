"""Multi-process sharding (world_size 2, gloo, CPU).

The per-rank device evaluation is replaced by the numpy mirror of the kernels
(tests/bytecode_ref.py) so that the sharding, the collectives and the result
assembly run here exactly as on the GPU box; results must equal the
single-process evaluation (population sharding: identical; case sharding:
within the fp64 tolerance, exceptions and their first-case order exact)."""
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import bytecode_ref as ref
from deap_amd import _lib, configs, datasets, gp
from deap_amd.distributed import (CaseSharded, PopulationSharded,
                                  balanced_ranges, shard_range)
from deap_amd.evaluator import BooleanHits, SymbRegMSE, pack_bitplanes
from deap_amd.flatten import Flattener, Machine


class CpuLocal(object):
    """Stand-in for GPUEvaluator with the same flatten/run_batch contract."""

    def __init__(self, pset, spec):
        self.spec = spec
        self.flattener = Flattener(pset, spec.machine)

    def flatten(self, inds):
        return self.flattener.flatten(inds)

    def run_batch(self, batch):
        n = len(batch)
        hi = np.zeros(n)
        lo = np.zeros(n)
        err = np.full(n, _lib.GPE_NO_ERROR, dtype=np.uint64)
        flags = np.zeros(n, dtype=np.uint32)
        for i in range(n):
            code = batch.code[batch.offsets[i]:batch.offsets[i + 1]]
            if self.spec.machine == Machine.B:
                T = ref.run_b(code, self.spec.planes)
                agree = ~(T ^ self.spec.out_plane)
                bits = np.unpackbits(agree.view(np.uint8),
                                     bitorder="little")[:self.spec.n_cases]
                hi[i] = bits.sum()
                continue
            T, verr = ref.run_f(code, self.spec.X)
            d = T.copy()
            for t in self.spec.terms:
                d = d - t
            with np.errstate(all="ignore"):
                sq = d * d
            ovf = np.isfinite(d) & np.isinf(sq)
            bad = np.nonzero(verr | ovf)[0]
            if len(bad):
                c = int(bad[0])
                err[i] = (c << 2) | (1 if verr[c] else 2)
            if not np.isfinite(d).all():
                flags[i] = 1
            fin = np.isfinite(sq)
            hi[i] = math.fsum(sq[fin].tolist()) if fin.all() else \
                (np.nan if np.isnan(sq).any() else np.inf)
        return hi, lo, err, flags, None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, kind, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if kind == "case":
            pset = configs.pset_for("symreg10")
            X, Y = datasets.symreg10_cases(999, 3)
            lo, hi = shard_range(X.shape[1], rank, world)
            local = CpuLocal(pset, SymbRegMSE(X[:, lo:hi], Y[:, lo:hi]))
            ev = CaseSharded(local, X.shape[1], lo,
                             reduce="allgather" if rank >= 0 else None)
            pop = configs.population(pset, "half", 60, 5, 2, 5)
            res = ev.evaluate(pop)
            ev.reduce = "allreduce"
            res2 = ev.evaluate(pop)
        else:
            pset = configs.pset_for("parity6")
            ins, outs = datasets.parity6_table()
            local = CpuLocal(pset, BooleanHits(ins, outs))
            pop = configs.population(pset, "full", 101, 6, 3, 5)
            res = PopulationSharded(local).evaluate(pop)
            res2 = res
        q.put((rank, [r if not isinstance(r, BaseException)
                      else type(r).__name__ for r in res],
               [r if not isinstance(r, BaseException)
                else type(r).__name__ for r in res2]))
    finally:
        dist.destroy_process_group()


def _run(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, q))
             for r in range(2)]
    for p in procs:
        p.start()
    out = dict()
    for _ in procs:
        rank, a, b = q.get(timeout=240)
        out[rank] = (a, b)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_case_sharded_equals_single_process():
    out = _run("case")
    pset = configs.pset_for("symreg10")
    X, Y = datasets.symreg10_cases(999, 3)
    local = CpuLocal(pset, SymbRegMSE(X, Y))
    pop = configs.population(pset, "half", 60, 5, 2, 5)
    b = local.flatten(pop)
    h, l, e, f, _ = local.run_batch(b)
    single = [local.spec.finish(i, h[i], l[i], e[i], f[i])
              for i in range(len(pop))]
    for rank in (0, 1):
        for variant in out[rank]:
            assert len(variant) == len(single)
            for a, s in zip(variant, single):
                if isinstance(s, BaseException):
                    assert a == type(s).__name__
                else:
                    a = a[0]
                    s = s[0]
                    assert (a == s) or abs(a - s) <= 1e-12 * abs(s) or \
                        (math.isnan(a) and math.isnan(s))


def test_population_sharded_is_bit_identical():
    out = _run("pop")
    pset = configs.pset_for("parity6")
    ins, outs = datasets.parity6_table()
    pop = configs.population(pset, "full", 101, 6, 3, 5)
    exp = []
    for t in pop:
        fn = gp.compile(t, pset)
        exp.append((int(sum(fn(*ins[:, c]) == outs[c]
                            for c in range(64))),))
    assert out[0][0] == exp and out[1][0] == exp


class _FinishOnly(object):
    """A user spec with ``finish`` and no ``finish_all``."""
    mode = _lib.GPE_MODE_HITS_BITS

    def finish(self, i, hi, lo, err, flags):
        return (int(hi),)


class _GatheredCtx(object):
    """gpe_run_gathered's result layout without a device: rank r's program
    i at r * width + i, the padding zero."""

    def __init__(self, ranges, width):
        self.ranges, self.width = ranges, width

    def run_gathered(self, mode, width, world, tags=None, want=None):
        m = width * world
        hi = np.zeros(m)
        for r, (a, b) in enumerate(self.ranges):
            hi[r * width:r * width + b - a] = np.arange(a, b) + 100
        return (hi, np.zeros(m), np.zeros(m, np.uint64),
                np.zeros(m, np.uint32))


@pytest.mark.parametrize("ranges", [[(0, 6)], [(0, 3), (3, 6)],
                                    [(0, 4), (4, 6)]])
def test_gathered_results_with_finish_only_spec(ranges):
    """a spec without finish_all, every slice at the full width
    (world 1, or an even split), must not depend on the padding index."""
    local = type("L", (), {"spec": _FinishOnly()})()
    width = max(b - a for a, b in ranges)
    batch = type("B", (), {"err": np.zeros(6, np.uint8)})()
    ev = PopulationSharded(local)
    out = ev._evaluate_native(_GatheredCtx(ranges, width), list(range(6)),
                              ranges, width, batch)
    assert out == [(100 + i,) for i in range(6)]


def test_balanced_ranges_cover_and_balance():
    rng = np.random.default_rng(0)
    lens = rng.integers(1, 300, size=1000)
    for world in (1, 2, 3, 8):
        rs = balanced_ranges(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == 1000
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        tot = [lens[a:b].sum() for a, b in rs]
        assert max(tot) - min(tot) <= 2 * lens.max()
    assert shard_range(10, 0, 3) == (0, 3) and shard_range(10, 2, 3) == (6, 10)
