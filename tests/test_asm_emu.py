"""The exact cores' generated sin/cos handlers, executed on the CPU
(tests/asm_emu.py) against the host libm — the reference's math.sin/cos
(glibc 2.35) — bit for bit, without a GPU.

Covers every range of s_sin.c (|x| < 0.126 TAYLOR_SIN, < 0.855469,
< 2.426265, reduce_sincos below 105414350, __branred beyond), their edges,
signed zeros, waves mixing all of them in one chain or in one lane group,
and waves whose chains differ (the per-chain EXEC masks).  The GPU twin of
this test is test_gpu.py::test_exact_asm_core_sin_cos_are_the_host_libm.
"""
import math
import os

import numpy as np
import pytest

import asm_emu

EDGES = np.array([0.0, 2.0 ** -26, 2.0 ** -27, 0.126, 0.855469, 2.426265,
                  105414350.0, 1e-300, 5e-324, 2.0 ** 40, 1e22, 1e300,
                  math.pi / 2, math.pi, 0.78539816339744828])


def _waves(rng, n):
    kinds = []
    for i in range(n):
        t = i % 6
        if t == 0:           # all ranges shuffled
            x = np.concatenate([rng.uniform(-0.2, 0.2, 32), rng.uniform(-3, 3, 32),
                                rng.uniform(-1e4, 1e4, 32), rng.uniform(-1, 1, 32)])
            rng.shuffle(x)
        elif t == 1:         # chain 0 small only, chain 1 mixed
            x = np.concatenate([rng.uniform(-0.85, 0.85, 64), rng.uniform(-5, 5, 64)])
        elif t == 2:         # chain 0 mixed, chain 1 small only
            x = np.concatenate([rng.uniform(-5, 5, 64), rng.uniform(-0.85, 0.85, 64)])
        elif t == 3:         # __branred lanes in both chains (the slow path)
            x = rng.uniform(-3, 3, 128)
            x[rng.integers(0, 128, 6)] = np.ldexp(rng.random(6), rng.integers(27, 1024, 6))
        elif t == 4:         # edges, scaled by a few ulps, both signs
            e = EDGES[rng.integers(0, len(EDGES), 128)]
            x = e * (1 + rng.integers(-4, 5, 128) * 2.0 ** -52)
            x *= np.where(rng.random(128) < 0.5, -1.0, 1.0)
        else:                # tiny and huge magnitudes
            x = np.ldexp(rng.random(128), rng.integers(-1075, 1024, 128))
            x *= np.where(rng.random(128) < 0.5, -1.0, 1.0)
        kinds.append(x)
    return kinds


@pytest.mark.parametrize("suffix", ["_exact", "_exact_deep"])
@pytest.mark.parametrize("which", ["SIN", "COS"])
def test_generated_exact_handler_is_the_host_libm(which, suffix):
    if not os.path.exists(os.path.join(asm_emu.CSRC, "gp_asm_core%s.inc" % suffix)):
        pytest.skip("cores not generated (python -m deap_amd.build)")
    f = math.sin if which == "SIN" else math.cos
    rng = np.random.default_rng(606 + (which == "COS") + 2 * (suffix == "_exact_deep"))
    lines = asm_emu.handler_lines(which, suffix)
    for x in _waves(rng, 36):
        x = np.concatenate([x[:-2], [0.0, -0.0]]) if rng.random() < 0.2 else x
        y, vred = asm_emu.run_handler(which, x, suffix, lines)
        ref = np.array([f(v) for v in x.tolist()])
        bad = y.view(np.uint64) != ref.view(np.uint64)
        assert not bad.any(), (x[bad][:4], y[bad][:4], ref[bad][:4])
        # VRED: the running max of |x|.hi (the C++ pass's inf/nan test)
        hx = (x.view(np.uint64) >> 32).astype(np.uint32) & 0x7FFFFFFF
        assert (vred == np.maximum(hx[:64], hx[64:])).all()
