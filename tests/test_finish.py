"""The vectorised fitness finishing (finish_all) returns exactly what the
per-individual finish returns, exceptions included (host only, no GPU)."""
import math

import numpy as np
import pytest

from deap_amd import _lib
from deap_amd.evaluator import (BooleanHits, SymbRegMSE, SymbRegNumpySSE,
                                SymbRegSumSSE, TypedBoolHits)


def arrays(n, seed):
    rng = np.random.default_rng(seed)
    hi = rng.random(n) * 10.0 ** rng.integers(-300, 300, n)
    hi[rng.random(n) < 0.05] = np.inf
    hi[rng.random(n) < 0.05] = np.nan
    lo = hi * rng.standard_normal(n) * 2.0 ** -60
    lo[~np.isfinite(lo)] = 0.0
    err = np.full(n, _lib.GPE_NO_ERROR, dtype=np.uint64)
    pick = rng.random(n) < 0.1
    err[pick] = (rng.integers(0, 1000, pick.sum()).astype(np.uint64) << 2) \
        | rng.integers(1, 3, pick.sum()).astype(np.uint64)
    flags = rng.integers(0, 8, n).astype(np.uint32)
    return hi, lo, err, flags


def same(a, b):
    if isinstance(a, BaseException):
        return type(a) is type(b) and a.args == b.args
    return len(a) == len(b) and all(
        x == y or (isinstance(x, float) and math.isnan(x) and math.isnan(y))
        for x, y in zip(a, b))


@pytest.mark.parametrize("spec", [
    SymbRegMSE(np.zeros((1, 20)), np.zeros((1, 20))),
    SymbRegNumpySSE(np.zeros((1, 7)), np.zeros((1, 7))),
    SymbRegSumSSE(np.zeros((1, 20)), np.zeros((1, 20))),
    BooleanHits(np.zeros((2, 64), np.uint8), np.zeros(64, np.uint8)),
    TypedBoolHits(np.zeros((3, 10)), np.zeros(10))])
def test_finish_all_matches_finish(spec):
    hi, lo, err, flags = arrays(5000, 1)
    if isinstance(spec, (BooleanHits, TypedBoolHits)):
        hi = np.floor(np.random.default_rng(2).random(5000) * 5000)
    got = spec.finish_all(hi, lo, err, flags)
    for i in range(len(hi)):
        assert same(got[i], spec.finish(i, hi[i], lo[i], err[i], flags[i])), i
