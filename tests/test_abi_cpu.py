"""CPU-side checks of the product library: it builds for gfx950, loads,
exports every entry point of include/mi_lp.h, keeps the ctypes struct layout
in sync with the C header, and refuses to run without a GPU (no fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

from mi_glop import abi, engine

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_loads_and_exports_header_symbols():
    L = engine.lib()
    header = open(os.path.join(REPO, "include", "mi_lp.h")).read()
    declared = sorted(set(re.findall(r"\b(mi_(?:lp|glop|mps|exchange|presolve)_[a-z_]+)\(", header)))
    assert declared == sorted(abi.EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (mi_\w+)", out))
    assert exported == set(declared)


def test_code_object_targets_gfx950():
    blob = open(engine.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_default_params_match_c_defaults():
    L = engine.lib()
    c = abi.MiGlopParams()
    L.mi_glop_params_default(ctypes.byref(c))
    py = abi.default_params()
    for name, _ in abi.MiGlopParams._fields_:
        assert getattr(c, name) == getattr(py, name), name


def test_no_gpu_means_loud_failure():
    if engine.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(engine.EngineUnavailable):
        engine.LpHandle()
