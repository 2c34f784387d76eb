"""ctypes binding of the CPU oracle (oracle/build/liboracle_glop.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker, never the product.
"""
import ctypes
import os
import subprocess

import numpy as np

from mi_glop import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle_glop.so")

_libs = {}


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib(variant="glop"):
    """variant "glop": the oracle. "sdual": the same oracle with the device
    dual segment's host restatement (or-tools_amd/csrc/sdual) in its dual loop,
    a test-only build that the CPU checks compare with the oracle."""
    if variant not in _libs:
        path = os.path.join(ORACLE_DIR, "build", f"liboracle_{variant}.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_lp_create.restype = ctypes.c_void_p
        L.oracle_lp_destroy.argtypes = [ctypes.c_void_p]
        vp = ctypes.c_void_p
        L.oracle_lp_set_params.argtypes = [vp, ctypes.POINTER(abi.MiGlopParams)]
        L.oracle_lp_load.argtypes = [vp, ctypes.c_int32, ctypes.c_int32] + \
            [ctypes.c_void_p] * 8 + [ctypes.c_double, ctypes.c_double, ctypes.c_int32]
        L.oracle_lp_solve.argtypes = [vp, ctypes.c_void_p, ctypes.POINTER(abi.MiLpResult)]
        for name in ["oracle_lp_get_primal", "oracle_lp_get_reduced_costs",
                     "oracle_lp_get_duals", "oracle_lp_get_activities",
                     "oracle_lp_get_basis", "oracle_lp_get_state",
                     "oracle_lp_get_primal_ray", "oracle_lp_get_dual_ray"]:
            getattr(L, name).argtypes = [vp, ctypes.c_void_p]
        L.oracle_lp_get_statuses.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_lp_load_basis_state.argtypes = [vp, ctypes.c_void_p, ctypes.c_int32]
        L.oracle_lp_clear_basis_state.argtypes = [vp]
        L.oracle_lp_notify_matrix_unchanged.argtypes = [vp]
        L.oracle_lp_record_iteration_times.argtypes = [vp, ctypes.c_int32]
        L.oracle_lp_get_iteration_times.argtypes = [vp, ctypes.c_void_p, ctypes.c_int64]
        L.oracle_lp_set_variable_bounds.argtypes = [vp, vp, vp]
        L.oracle_lp_batch_solve_bounds.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp,
                                                   vp, ctypes.c_int32,
                                                   ctypes.POINTER(abi.MiLpResult)]
        L.oracle_lp_get_iteration_times.restype = ctypes.c_int64
        L.oracle_lp_notify_matrix_changed.argtypes = [vp]
        L.oracle_lp_set_starting_variable_values.argtypes = [vp, vp, ctypes.c_int32]
        L.oracle_lp_set_integrality_scale.argtypes = [vp, ctypes.c_int32, ctypes.c_double]
        L.oracle_lp_clear_integrality_scales.argtypes = [vp]
        L.oracle_lp_objective_limit_reached.argtypes = [vp, vp]
        L.oracle_lp_get_unit_row_left_inverse.argtypes = [vp, ctypes.c_int32, vp, vp, vp]
        L.oracle_lp_compute_dictionary.argtypes = [vp, vp, ctypes.c_int32, vp]
        L.oracle_lp_get_dictionary.argtypes = [vp, vp, vp, vp]
        _libs[variant] = L
    return _libs[variant]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleLp:
    """Same surface as mi_glop.engine.LpHandle, CPU restatement behind it."""

    def __init__(self, params=None, variant="glop"):
        self._L = lib(variant)
        self.h = ctypes.c_void_p(self._L.oracle_lp_create())
        self.params = params or abi.default_params()
        self.lp = None

    def __del__(self):
        if getattr(self, "h", None):
            self._L.oracle_lp_destroy(self.h)
            self.h = None

    def set_params(self, params):
        self.params = params

    def load(self, lp):
        self.lp = lp
        self._keep = [np.ascontiguousarray(x, dtype=t) for x, t in (
            (lp.col_starts, np.int64), (lp.row_idx, np.int32), (lp.vals, np.float64),
            (lp.col_lb, np.float64), (lp.col_ub, np.float64), (lp.row_lb, np.float64),
            (lp.row_ub, np.float64), (lp.obj, np.float64))]
        cs, ri, v, clb, cub, rlb, rub, ob = self._keep
        self._L.oracle_lp_load(self.h, lp.m, lp.n, _p(cs), _p(ri), _p(v), _p(clb),
                               _p(cub), _p(rlb), _p(rub), _p(ob), lp.obj_offset,
                               lp.obj_scale, int(lp.maximize))

    def set_variable_bounds(self, col_lb, col_ub):
        self._lbk = np.ascontiguousarray(col_lb, dtype=np.float64)
        self._ubk = np.ascontiguousarray(col_ub, dtype=np.float64)
        self._L.oracle_lp_set_variable_bounds(self.h, _p(self._lbk), _p(self._ubk))

    def load_basis_state(self, state):
        st = np.ascontiguousarray(state, dtype=np.int8)
        self._L.oracle_lp_load_basis_state(self.h, _p(st), len(st))

    def clear_basis_state(self):
        self._L.oracle_lp_clear_basis_state(self.h)

    def notify_matrix_unchanged(self):
        self._L.oracle_lp_notify_matrix_unchanged(self.h)

    def record_iteration_times(self, on=True):
        self._L.oracle_lp_record_iteration_times(self.h, int(on))

    def iteration_times(self):
        n = self._L.oracle_lp_get_iteration_times(self.h, None, 0)
        out = np.zeros(n)
        self._L.oracle_lp_get_iteration_times(self.h, _p(out), n)
        return out

    def solve(self):
        self._L.oracle_lp_set_params(self.h, ctypes.byref(self.params))
        r = abi.MiLpResult()
        self._L.oracle_lp_solve(self.h, None, ctypes.byref(r))
        return r

    def _get(self, fn, n, dtype):
        out = np.zeros(n, dtype=dtype)
        getattr(self._L, fn)(self.h, _p(out))
        return out

    def primal(self):
        return self._get("oracle_lp_get_primal", self.lp.n, np.float64)

    def reduced_costs(self):
        return self._get("oracle_lp_get_reduced_costs", self.lp.n, np.float64)

    def duals(self):
        return self._get("oracle_lp_get_duals", self.lp.m, np.float64)

    def activities(self):
        return self._get("oracle_lp_get_activities", self.lp.m, np.float64)

    def basis(self):
        return self._get("oracle_lp_get_basis", self.lp.m, np.int32)

    def state(self):
        return self._get("oracle_lp_get_state", self.lp.n + self.lp.m, np.int8)

    def statuses(self):
        var = np.zeros(self.lp.n, np.int8)
        cons = np.zeros(self.lp.m, np.int8)
        self._L.oracle_lp_get_statuses(self.h, _p(var), _p(cons))
        return var, cons

    def primal_ray(self):
        return self._get("oracle_lp_get_primal_ray", self.lp.n + self.lp.m, np.float64)

    def dual_ray(self):
        return self._get("oracle_lp_get_dual_ray", self.lp.m, np.float64)

    def _call(self, name, *args):
        getattr(self._L, "oracle_lp_" + name)(self.h, *args)

    # --- CP-SAT boundary (include/mi_lp.h) ---------------------------------
    def notify_matrix_changed(self):
        self._call("notify_matrix_changed")

    def set_starting_variable_values(self, values):
        self._start_values = np.ascontiguousarray(values, dtype=np.float64)
        self._call("set_starting_variable_values", _p(self._start_values),
                   len(self._start_values))

    def set_integrality_scale(self, col, scale):
        self._call("set_integrality_scale", int(col), ctypes.c_double(scale))

    def clear_integrality_scales(self):
        self._call("clear_integrality_scales")

    def objective_limit_reached(self):
        r = ctypes.c_int32()
        self._call("objective_limit_reached", ctypes.byref(r))
        return bool(r.value)

    def unit_row_left_inverse(self, row):
        """(dense values[m], non-zero rows) of e_row^T B^-1."""
        vals = np.zeros(self.lp.m, np.float64)
        nz = np.zeros(self.lp.m, np.int32)
        cnt = ctypes.c_int32()
        self._call("get_unit_row_left_inverse", int(row), _p(vals), _p(nz), ctypes.byref(cnt))
        return vals, nz[:cnt.value].copy()

    def dictionary(self, column_scales=None):
        """B^-1 A as (row_starts[m+1], cols, values), rows in basis order."""
        nnz = ctypes.c_int64()
        if column_scales is None:
            self._call("compute_dictionary", None, 0, ctypes.byref(nnz))
        else:
            sc = np.ascontiguousarray(column_scales, dtype=np.float64)
            self._call("compute_dictionary", _p(sc), len(sc), ctypes.byref(nnz))
        starts = np.zeros(self.lp.m + 1, np.int64)
        cols = np.zeros(max(1, nnz.value), np.int32)
        vals = np.zeros(max(1, nnz.value), np.float64)
        self._call("get_dictionary", _p(starts), _p(cols), _p(vals))
        return starts, cols[:nnz.value], vals[:nnz.value]


def batch_solve_bounds(workers, lbs, ubs, warm_state=None):
    """CPU baseline / checker of engine.batch_solve_bounds (one thread per
    oracle worker, shared LP counter)."""
    L = workers[0]._L
    for w in workers:
        L.oracle_lp_set_params(w.h, ctypes.byref(w.params))
    lbs = np.ascontiguousarray(lbs, dtype=np.float64)
    ubs = np.ascontiguousarray(ubs, dtype=np.float64)
    count = lbs.shape[0]
    arr = (ctypes.c_void_p * len(workers))(*[w.h.value for w in workers])
    res = (abi.MiLpResult * count)()
    ws = None if warm_state is None else np.ascontiguousarray(warm_state, dtype=np.int8)
    L.oracle_lp_batch_solve_bounds(arr, len(workers), count, _p(lbs), _p(ubs),
                                   None if ws is None else _p(ws),
                                   0 if ws is None else len(ws), res)
    return list(res)
