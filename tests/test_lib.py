"""The C-ABI library builds, loads on a GPU-less host, and exports every
symbol include/gpeval.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

from conftest import REPO
from deap_amd import _lib, build


def header_symbols():
    with open(os.path.join(REPO, "include", "gpeval.h")) as fh:
        text = fh.read()
    return sorted(set(re.findall(r"\b(gpe_[a-z_]+)\s*\(", text)))


def test_library_exports_header_symbols():
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES)


def test_missing_library_is_loud(tmp_path):
    import pytest
    saved = _lib._lib
    _lib._lib = None
    try:
        with pytest.raises(_lib.GpeError):
            _lib.load(str(tmp_path / "nope.so"))
    finally:
        _lib._lib = saved


def test_library_is_gfx950_code_object():
    build.build()
    with open(_lib.LIB_PATH, "rb") as fh:
        blob = fh.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_kernel_sin_cos_are_nearly_correctly_rounded():
    """The kernels' sin/cos (host-compiled twin, bit-identical code) must be
    correctly rounded in >= 99.8 % of calls — at least as often as glibc's
    math.sin/cos, which the reference calls — so device and reference differ
    only where one of them misrounds."""
    import math
    import mpmath
    import numpy as np
    build.build()
    mpmath.mp.prec = 160
    rng = np.random.default_rng(7)
    for fn, f in ((0, mpmath.sin), (1, mpmath.cos)):
        for lo, hi in ((-1, 1), (-60, 60), (-3e4, 3e4)):
            x = rng.uniform(lo, hi, 3000)
            y = _lib.host_math(fn, x)
            cr = np.array([float(f(mpmath.mpf(v))) for v in x])
            assert (y != cr).mean() <= 0.002
            assert (np.abs(y - cr) <= np.spacing(np.abs(cr))).all()
        # the doubles nearest k*pi/32: tiny residuals, where the reduction's
        # relative accuracy decides (within 1 ulp up to 2^20)
        k = rng.integers(-10 ** 7, 10 ** 7, 1500)
        x = np.array([float(int(v) * mpmath.pi / 32) for v in k])
        y = _lib.host_math(fn, x)
        cr = np.array([float(f(mpmath.mpf(v))) for v in x])
        assert (np.abs(y - cr) <= np.spacing(np.abs(cr))).all()
        assert (y != cr).mean() <= 0.002
    x = np.array([0.0, -0.0, 1e-300, 5e-324, 1.5707963267948966, 1e6, 1e300])
    for fn, f in ((0, math.sin), (1, math.cos)):
        y = _lib.host_math(fn, x)
        exp = np.array([f(v) for v in x])
        assert np.allclose(y, exp, rtol=2.3e-16, atol=0)
        assert np.signbit(y[1]) == np.signbit(exp[1])
    y = _lib.host_math(0, np.array([np.inf, np.nan]))
    assert np.isnan(y).all()


def test_numpy_order_row_sum_is_bit_identical_to_numpy_sum():
    """GPE_MODE_SSE_NUMPY's reduction (host twin, same code as the device
    kernel np_sum_rows) reproduces numpy.sum bit for bit: pairwise blocks of
    128 inside 8192-element buffer chunks, nan/inf/overflow included."""
    import numpy as np
    build.build()
    rng = np.random.default_rng(3)
    for t in range(200):
        n = int(rng.integers(1, 40000)) if t > 4 else (1, 7, 8, 129, 8193)[t]
        x = (rng.standard_normal(n) * np.exp(rng.uniform(-30, 30, n))) ** 2
        if t % 7 == 0:
            x[rng.integers(0, n)] = np.inf
        if t % 11 == 0:
            x[rng.integers(0, n)] = np.nan
        if t % 13 == 0:
            x[:] = 1e300                         # overflow of finite terms
        a = np.sum(x)
        b = _lib.host_np_sum(x)[0]
        assert a == b or (np.isnan(a) and np.isnan(b)), (n, a, b)
    rows = rng.random((5, 10000))
    assert np.array_equal(_lib.host_np_sum(rows), rows.sum(axis=1))


def test_fp32_mode_sin_cos_within_one_ulp():
    """gp_trig32 (fp32 mode; host twin of the device code) is within 1 ulp
    (fp32) of the correctly rounded value below 2^20."""
    import mpmath
    import numpy as np
    build.build()
    mpmath.mp.prec = 100
    rng = np.random.default_rng(11)
    for lo, hi in ((-1, 1), (-100, 100), (-1e5, 1e5)):
        x = rng.uniform(lo, hi, 2000).astype(np.float32).astype(np.float64)
        for fn, f in ((3, mpmath.sin), (4, mpmath.cos)):
            y = _lib.host_math(fn, x).astype(np.float32)
            ref = np.array([float(f(mpmath.mpf(v))) for v in x],
                           dtype=np.float32)
            err = np.abs(y.astype(np.float64) - ref) / \
                np.spacing(np.abs(ref)).astype(np.float64)
            assert err.max() <= 1.0


def test_glibc_restatement_is_the_host_libm_bit_for_bit():
    """glibc_sin/glibc_cos (gpeval.hip: glibc 2.35 s_sin.c + branred.c
    restated, used by gp_trig beyond 2^40 and by the redo pass) return the
    host libm's bits — the reference's math.sin/cos — over the whole double
    range: every binade, subnormals, the branch points of __sin/__cos,
    signed zeros, inf and nan."""
    import math
    import numpy as np
    build.build()
    rng = np.random.default_rng(11)
    n = 200000
    parts = [np.ldexp(rng.random(n), rng.integers(-1075, 1024, n)),
             rng.uniform(-8, 8, n),
             np.ldexp(rng.random(n), rng.integers(-30, 90, n))]
    edges = np.array([2.0 ** -26, 2.0 ** -27, 0.126, 0.855469, 2.426265,
                      105414350.0, 2.0 ** 40, 1e300, 5e-324])
    parts.append((edges[:, None] * (1 + np.arange(-64, 65) * 2.0 ** -50))
                 .ravel())
    x = np.concatenate(parts)
    x = np.concatenate([x, -x, [0.0, -0.0, np.inf, -np.inf, np.nan]])
    for fn, f in ((5, math.sin), (6, math.cos), (7, math.sin), (8, math.cos)):
        y = _lib.host_math(fn, x)
        with np.errstate(invalid="ignore"):
            ref = np.array([f(v) if math.isfinite(v) else v - v
                            for v in x.tolist()])
        same = (y.view(np.uint64) == ref.view(np.uint64)) | \
            (np.isnan(y) & np.isnan(ref))
        assert same.all(), (fn, x[~same][:5])


def test_collective_waits_are_bounded():
    """VERDICT r4 #3b: a wait on a stream holding RCCL collectives polls with
    a deadline (GPE_COMM_TIMEOUT_S) instead of blocking; on expiry the call
    fails with GPE_E_COMM naming the collective and the rank (no HIP call
    here: a fake stream that stays busy)."""
    rc, msg = _lib.debug_bounded_wait(0.05, -1)          # never completes
    assert rc == _lib.GPE_E_COMM
    assert "not complete after" in msg and "rank 0 of 1" in msg \
        and "aborted" in msg, msg
    rc, msg = _lib.debug_bounded_wait(5.0, 1000)          # completes in time
    assert rc == 0 and msg == ""


def test_translation_unit_headers_are_tracked_and_included():
    """gpeval.hip's parts live in headers (DESIGN §3 "Source layout"): every
    header the TU includes from csrc/ is one build.py rebuilds on and
    scripts/build_variant.sh copies, so no edit can go unbuilt or leave a
    variant build without it."""
    csrc = os.path.join(REPO, "deap_amd", "csrc")
    src = open(os.path.join(csrc, "gpeval.hip")).read()
    included = set(re.findall(r'^#include "([a-z_]+\.h)"', src, re.M))
    generated = {h for h in included if h.startswith("gp_asm_layout")}
    parts = included - generated
    assert {"trig_dev.h", "exact_int.h", "planner.h", "ctx.h"} <= parts
    assert parts <= set(build.LIB_HEADERS), parts - set(build.LIB_HEADERS)
    variant = open(os.path.join(REPO, "scripts", "build_variant.sh")).read()
    for h in build.LIB_HEADERS:
        assert os.path.exists(os.path.join(csrc, h)), h
        assert "deap_amd/csrc/" + h in variant, h
