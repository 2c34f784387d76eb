"""MPS files into LinearProgram, through the engine library's reader
(include/mi_lp.h mi_mps_*, a restatement of glop::MPSReader: ortools/lp_data/
mps_reader.h:39-60 and mps_reader_template.h). Pure host code: works without
a GPU. Integer markers are parsed; the LinearProgram is their relaxation,
with the 0/1 default bounds upstream gives integer-section columns."""
import ctypes
import os

import numpy as np

from . import engine
from .lp import LinearProgram

AUTO, FREE, FIXED = 0, 1, 2
FORMAT_NAMES = {FREE: "free", FIXED: "fixed"}


class MpsError(ValueError):
    """absl::InvalidArgumentError of the upstream reader."""


def _bind(L):
    if getattr(L, "_mps_bound", False):
        return L
    vp = ctypes.c_void_p
    L.mi_mps_read_file.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.POINTER(vp),
                                   ctypes.POINTER(ctypes.c_int32)]
    L.mi_mps_parse_string.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.POINTER(vp),
                                      ctypes.POINTER(ctypes.c_int32)]
    L.mi_mps_error.argtypes = [vp]
    L.mi_mps_error.restype = ctypes.c_char_p
    L.mi_mps_dims.argtypes = [vp, ctypes.POINTER(ctypes.c_int32),
                              ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]
    L.mi_mps_get.argtypes = [vp] * 10 + [ctypes.POINTER(ctypes.c_int32), vp]
    L.mi_mps_name.argtypes = [vp]
    L.mi_mps_name.restype = ctypes.c_char_p
    L.mi_mps_col_name.argtypes = [vp, ctypes.c_int32]
    L.mi_mps_col_name.restype = ctypes.c_char_p
    L.mi_mps_row_name.argtypes = [vp, ctypes.c_int32]
    L.mi_mps_row_name.restype = ctypes.c_char_p
    L.mi_mps_free.argtypes = [vp]
    L._mps_bound = True
    return L


def _to_lp(L, model, with_names):
    m = ctypes.c_int32()
    n = ctypes.c_int32()
    nnz = ctypes.c_int64()
    L.mi_mps_dims(model, ctypes.byref(m), ctypes.byref(n), ctypes.byref(nnz))
    m, n, nnz = m.value, n.value, nnz.value
    cs = np.zeros(n + 1, np.int64)
    ri = np.zeros(max(nnz, 1), np.int32)
    va = np.zeros(max(nnz, 1), np.float64)
    col_lb, col_ub, obj = (np.zeros(n) for _ in range(3))
    row_lb, row_ub = np.zeros(m), np.zeros(m)
    offset = ctypes.c_double()
    maximize = ctypes.c_int32()
    is_int = np.zeros(max(n, 1), np.int8)
    P = engine._p
    L.mi_mps_get(model, P(cs), P(ri), P(va), P(col_lb), P(col_ub), P(row_lb), P(row_ub),
                 P(obj), ctypes.cast(ctypes.byref(offset), ctypes.c_void_p),
                 ctypes.byref(maximize), P(is_int))
    lp = LinearProgram(m, n, cs, ri[:nnz], va[:nnz], col_lb, col_ub, row_lb, row_ub, obj,
                       obj_offset=offset.value, maximize=bool(maximize.value),
                       name=L.mi_mps_name(model).decode() or "mps")
    lp.is_integer = is_int[:n].astype(bool)
    if with_names:
        lp.col_names = [L.mi_mps_col_name(model, j).decode() for j in range(n)]
        lp.row_names = [L.mi_mps_row_name(model, i).decode() for i in range(m)]
    return lp


def _finish(L, rc, model, used, with_names):
    try:
        if rc != 0:
            raise MpsError(L.mi_mps_error(model).decode())
        lp = _to_lp(L, model, with_names)
        lp.mps_format = FORMAT_NAMES.get(used.value, "?")
        return lp
    finally:
        L.mi_mps_free(model)


def read_mps(path, fmt=AUTO, with_names=False):
    """MPSReader::ParseFile(path, LinearProgram*) -> LinearProgram."""
    L = _bind(engine.lib())
    model = ctypes.c_void_p()
    used = ctypes.c_int32()
    rc = L.mi_mps_read_file(os.fsencode(path), fmt, ctypes.byref(model), ctypes.byref(used))
    return _finish(L, rc, model, used, with_names)


def parse_mps(text, fmt=AUTO, with_names=False):
    """MPSReader::ParseString(text, LinearProgram*) -> LinearProgram."""
    L = _bind(engine.lib())
    model = ctypes.c_void_p()
    used = ctypes.c_int32()
    rc = L.mi_mps_parse_string(text.encode(), fmt, ctypes.byref(model), ctypes.byref(used))
    return _finish(L, rc, model, used, with_names)
