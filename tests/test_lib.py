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
