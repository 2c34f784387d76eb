"""ctypes binding of the MI355X engine (or-tools_amd/lib/libmi_lp.so).

This is the product path: every solve runs the HIP kernels. There is no CPU
fallback: if the library or a GPU is missing, creating a handle raises.
"""
import ctypes
import os
import subprocess

import numpy as np

from . import abi

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MI_LP_LIB") or os.path.join(PKG_DIR, "lib", "libmi_lp.so")

_lib = None


class EngineUnavailable(RuntimeError):
    pass


# mi_lp_allgather_fn (include/mi_lp.h): ctx, send, send_bytes, recv, recv_bytes.
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64))
# include/mi_lp.h mi_lp_simplex_fn: the LPSolver's simplex, supplied by the caller.
SIMPLEX_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                              *([ctypes.c_void_p] * 8), ctypes.c_double, ctypes.c_double,
                              ctypes.c_int32, ctypes.c_void_p, *([ctypes.c_void_p] * 4))


def build(jobs=8):
    """Compiles the engine for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", PKG_DIR], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable(
            f"{LIB_PATH} is missing: run `make -C or-tools_amd` (no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    L.mi_glop_params_default.argtypes = [ctypes.POINTER(abi.MiGlopParams)]
    L.mi_lp_device_count.restype = ctypes.c_int
    L.mi_lp_shutdown.restype = ctypes.c_int
    # Drain the engine's resident grids and join its service threads while
    # the HIP runtime is still up: Python's atexit runs before the C exit
    # handlers (the runtime's and a profiler's own teardown).
    import atexit
    atexit.register(_shutdown, L)
    # RCCL bound sharing (engine/comm.hip).
    L.mi_lp_comm_get_unique_id.argtypes = [vp]
    L.mi_lp_comm_create.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(vp)]
    L.mi_lp_comm_rank.argtypes = [vp]
    L.mi_lp_comm_size.argtypes = [vp]
    L.mi_lp_share_bound.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int32]
    L.mi_lp_comm_allreduce_device.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int32]
    L.mi_lp_comm_allgather_device.argtypes = [vp, vp, vp, ctypes.c_int64]
    L.mi_lp_comm_last_error.argtypes = [vp]
    L.mi_lp_comm_last_error.restype = ctypes.c_char_p
    L.mi_lp_comm_destroy.argtypes = [vp]
    L.mi_lp_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.mi_lp_destroy.argtypes = [vp]
    L.mi_lp_last_error.argtypes = [vp]
    L.mi_lp_last_error.restype = ctypes.c_char_p
    L.mi_lp_set_params.argtypes = [vp, ctypes.POINTER(abi.MiGlopParams)]
    L.mi_lp_load.argtypes = [vp, ctypes.c_int32, ctypes.c_int32] + [vp] * 8 + \
        [ctypes.c_double, ctypes.c_double, ctypes.c_int32]
    L.mi_lp_load_basis_state.argtypes = [vp, vp, ctypes.c_int32]
    L.mi_lp_clear_basis_state.argtypes = [vp]
    L.mi_lp_notify_matrix_unchanged.argtypes = [vp]
    L.mi_lp_solve.argtypes = [vp, vp, ctypes.POINTER(abi.MiLpResult)]
    for name in ["mi_lp_get_primal", "mi_lp_get_reduced_costs", "mi_lp_get_duals",
                 "mi_lp_get_activities", "mi_lp_get_basis", "mi_lp_get_state",
                 "mi_lp_get_primal_ray", "mi_lp_get_dual_ray",
                 "mi_lp_get_dual_ray_row_combination"]:
        getattr(L, name).argtypes = [vp, vp]
    L.mi_lp_get_statuses.argtypes = [vp, vp, vp]
    L.mi_lp_begin.argtypes = [vp, ctypes.c_int64]
    L.mi_lp_run_until.argtypes = [vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                                  ctypes.POINTER(ctypes.c_int64)]
    L.mi_lp_finish.argtypes = [vp, ctypes.POINTER(abi.MiLpResult)]
    L.mi_lp_stop.argtypes = [vp]
    L.mi_lp_get_kernel_stats.argtypes = [vp, ctypes.POINTER(abi.MiLpKernelStats)]
    L.mi_lp_reset_kernel_stats.argtypes = [vp]
    L.mi_lp_set_kernel_timing.argtypes = [vp, ctypes.c_int32]
    L.mi_lp_set_kernel_timing_ids.argtypes = [vp, ctypes.c_uint32]
    L.mi_lp_batch_solve.argtypes = [vp, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(abi.MiLpResult)]
    L.mi_lp_set_variable_bounds.argtypes = [vp, vp, vp]
    L.mi_lp_batch_solve_gpus.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.POINTER(abi.MiLpResult)]
    L.mi_lp_batch_solve_bounds.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp,
                                           ctypes.c_int32, ctypes.POINTER(abi.MiLpResult)]
    L.mi_lp_notify_matrix_changed.argtypes = [vp]
    L.mi_lp_set_starting_variable_values.argtypes = [vp, vp, ctypes.c_int32]
    L.mi_lp_set_integrality_scale.argtypes = [vp, ctypes.c_int32, ctypes.c_double]
    L.mi_lp_clear_integrality_scales.argtypes = [vp]
    L.mi_lp_record_iteration_times.argtypes = [vp, ctypes.c_int32]
    L.mi_lp_get_iteration_times.argtypes = [vp, vp, ctypes.c_int64]
    L.mi_lp_get_iteration_times.restype = ctypes.c_int64
    L.mi_lp_get_run_counters.argtypes = [vp, ctypes.POINTER(abi.MiLpRunCounters)]
    L.mi_lp_set_exchange.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, ALLGATHER_FN]
    L.mi_exchange_open.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int64, ctypes.POINTER(vp)]
    L.mi_exchange_allgather.argtypes = [vp, vp, ctypes.c_int64, vp, ctypes.POINTER(ctypes.c_int64)]
    L.mi_exchange_close.argtypes = [vp]
    L.mi_lp_objective_limit_reached.argtypes = [vp, vp]
    L.mi_lp_get_unit_row_left_inverse.argtypes = [vp, ctypes.c_int32, vp, vp, vp]
    L.mi_lp_compute_dictionary.argtypes = [vp, vp, ctypes.c_int32, vp]
    L.mi_lp_get_dictionary.argtypes = [vp, vp, vp, vp]
    L.mi_lp_solver_params_default.argtypes = [ctypes.POINTER(abi.MiLpSolverParams)]
    L.mi_lp_scale.argtypes = [ctypes.POINTER(abi.MiLpSolverParams), ctypes.c_int32,
                              ctypes.c_int32] + [vp] * 14
    L.mi_lp_solver_solve.argtypes = [vp, ctypes.POINTER(abi.MiLpSolverParams), ctypes.c_int32,
                                     ctypes.c_int32] + [vp] * 8 + [
        ctypes.c_double, ctypes.c_double, ctypes.c_int32, vp,
        ctypes.POINTER(abi.MiLpResult)] + [vp] * 6
    L.mi_lp_solver_solve_with.argtypes = [SIMPLEX_FN, vp, ctypes.POINTER(abi.MiLpSolverParams),
                                          ctypes.c_int32, ctypes.c_int32] + [vp] * 8 + [
        ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.POINTER(abi.MiLpResult)] + \
        [vp] * 6
    L.mi_presolve_create.restype = vp
    L.mi_presolve_destroy.argtypes = [vp]
    L.mi_presolve_run.argtypes = [vp, ctypes.POINTER(abi.MiLpSolverParams), ctypes.c_int32,
                                  ctypes.c_int32] + [vp] * 8 + [
        ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
    L.mi_presolve_dims.argtypes = [vp] + [vp] * 4
    L.mi_presolve_get.argtypes = [vp] + [vp] * 10
    L.mi_presolve_recover.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)] + [vp] * 8
    L.mi_presolve_num_passes.argtypes = [vp]
    L.mi_presolve_num_passes.restype = ctypes.c_int32
    L.mi_presolve_pass_name.argtypes = [vp, ctypes.c_int32]
    L.mi_presolve_pass_name.restype = ctypes.c_char_p
    _lib = L
    return L


_open_handles = None  # weakref.WeakSet of LpHandle, created with the first


def _shutdown(L):
    """Python exit: destroy the handles still open (their streams and device
    memory) and then the engine's shared device objects, before the HIP
    runtime and any profiler attached to it tear down."""
    if _open_handles is not None:
        for h in list(_open_handles):
            try:
                h.close()
            except Exception:  # noqa: BLE001 (exit path)
                pass
    L.mi_lp_shutdown()


def device_count():
    return lib().mi_lp_device_count()


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def allgather_callback(world, allgather):
    """A mi_lp_allgather_fn over a Python `allgather(data, sizes) -> bytes`.
    Failures return 1 (no exception may cross the C ABI; the engine then
    raises a DeviceError for the solve)."""
    def cb(_ctx, send, send_bytes, recv, recv_bytes):
        try:
            sizes = [int(recv_bytes[r]) for r in range(world)]
            data = ctypes.string_at(send, send_bytes) if send_bytes > 0 else b""
            out = allgather(data, sizes)
            if len(out) != sum(sizes):
                return 1
            if out:
                ctypes.memmove(recv, out, len(out))
            return 0
        except Exception:  # noqa: BLE001
            return 1
    return ALLGATHER_FN(cb)


class ShmExchange:
    """Same-node all-gather of host bytes in C++ (mi_exchange_open, engine/
    exchange.cc): the split's joins run without Python. Rank 0 creates the
    segment `name`, the other ranks attach (the call returns once all
    `world` ranks are attached). Needs no GPU."""

    def __init__(self, name, rank, world, slot_bytes=8 << 20):
        self._L = lib()
        x = ctypes.c_void_p()
        rc = self._L.mi_exchange_open(name.encode(), int(rank), int(world), int(slot_bytes),
                                      ctypes.byref(x))
        if rc != 0:
            raise RuntimeError(f"mi_exchange_open({name!r}, rank {rank}/{world}) failed with {rc}")
        self.x = x
        self.rank, self.world = int(rank), int(world)

    def allgather(self, data, sizes):
        """Every rank's bytes in rank order (sizes[r] from rank r)."""
        send = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
        recv = ctypes.create_string_buffer(max(1, sum(sizes)))
        arr = (ctypes.c_int64 * self.world)(*sizes)
        rc = self._L.mi_exchange_allgather(self.x, send, len(data), recv, arr)
        if rc != 0:
            raise RuntimeError(f"mi_exchange_allgather failed with {rc}")
        return recv.raw[:sum(sizes)]

    def function(self):
        """(ctx, mi_lp_allgather_fn) for mi_lp_set_exchange: the C function."""
        addr = ctypes.cast(self._L.mi_exchange_allgather, ctypes.c_void_p).value
        return self.x, ALLGATHER_FN(addr)

    def close(self):
        if getattr(self, "x", None):
            self._L.mi_exchange_close(self.x)
            self.x = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LpHandle:
    """One RevisedSimplex on one GPU (include/mi_lp.h)."""

    def __init__(self, params=None, device=0):
        self._L = lib()
        h = ctypes.c_void_p()
        rc = self._L.mi_lp_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise EngineUnavailable(f"mi_lp_create(device={device}) failed with {rc}: "
                                    "no usable MI355X (there is no CPU fallback)")
        self.h = h
        self.params = params or abi.default_params()
        self.lp = None
        global _open_handles
        if _open_handles is None:
            import weakref
            _open_handles = weakref.WeakSet()
        _open_handles.add(self)

    def close(self):
        if getattr(self, "h", None):
            self._L.mi_lp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self):
        msg = self._L.mi_lp_last_error(self.h)
        return msg.decode() if msg else ""

    def _check(self, rc, what):
        if rc != 0:
            msg = self._L.mi_lp_last_error(self.h)
            raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def set_params(self, params):
        self.params = params

    def load(self, lp):
        self.lp = lp
        self._keep = [np.ascontiguousarray(x, dtype=t) for x, t in (
            (lp.col_starts, np.int64), (lp.row_idx, np.int32), (lp.vals, np.float64),
            (lp.col_lb, np.float64), (lp.col_ub, np.float64), (lp.row_lb, np.float64),
            (lp.row_ub, np.float64), (lp.obj, np.float64))]
        cs, ri, v, clb, cub, rlb, rub, ob = self._keep
        self._check(self._L.mi_lp_load(self.h, lp.m, lp.n, _p(cs), _p(ri), _p(v),
                                       _p(clb), _p(cub), _p(rlb), _p(rub), _p(ob),
                                       lp.obj_offset, lp.obj_scale, int(lp.maximize)),
                    "mi_lp_load")

    def solve_lp(self, lp, solver_params=None, interrupt=None):
        """glop::LPSolver::SolveWithTimeLimit on this handle (mi_lp_solver_solve):
        scaling preprocessor, engine solve, RecoverSolution, solution values of
        the unscaled LP. Returns (result, dict of unscaled solution arrays)."""
        sp = solver_params or abi.default_solver_params()
        keep = [np.ascontiguousarray(x, dtype=t) for x, t in (
            (lp.col_starts, np.int64), (lp.row_idx, np.int32), (lp.vals, np.float64),
            (lp.col_lb, np.float64), (lp.col_ub, np.float64), (lp.row_lb, np.float64),
            (lp.row_ub, np.float64), (lp.obj, np.float64))]
        out = {"x": np.zeros(lp.n), "y": np.zeros(lp.m), "rc": np.zeros(lp.n),
               "act": np.zeros(lp.m), "vstat": np.zeros(lp.n, np.int8),
               "cstat": np.zeros(lp.m, np.int8)}
        r = abi.MiLpResult()
        flag = None if interrupt is None else _p(interrupt)
        self._push_params()
        rc = self._L.mi_lp_solver_solve(
            self.h, ctypes.byref(sp), lp.m, lp.n, *[_p(a) for a in keep], lp.obj_offset,
            lp.obj_scale, int(lp.maximize), flag, ctypes.byref(r),
            *[_p(out[k]) for k in ("x", "y", "rc", "act", "vstat", "cstat")])
        self._check(rc, "mi_lp_solver_solve")
        self.lp = None  # the handle now holds the scaled LP
        return r, out

    def set_variable_bounds(self, col_lb, col_ub):
        lb = np.ascontiguousarray(col_lb, dtype=np.float64)
        ub = np.ascontiguousarray(col_ub, dtype=np.float64)
        self._check(self._L.mi_lp_set_variable_bounds(self.h, _p(lb), _p(ub)),
                    "mi_lp_set_variable_bounds")

    def load_basis_state(self, state):
        st = np.ascontiguousarray(state, dtype=np.int8)
        self._check(self._L.mi_lp_load_basis_state(self.h, _p(st), len(st)),
                    "mi_lp_load_basis_state")

    def clear_basis_state(self):
        self._L.mi_lp_clear_basis_state(self.h)

    def notify_matrix_unchanged(self):
        self._L.mi_lp_notify_matrix_unchanged(self.h)

    def _push_params(self):
        self._check(self._L.mi_lp_set_params(self.h, ctypes.byref(self.params)),
                    "mi_lp_set_params")

    def solve(self):
        self._push_params()
        r = abi.MiLpResult()
        self._L.mi_lp_solve(self.h, None, ctypes.byref(r))
        if r.error_code == 100:
            raise EngineUnavailable(self._L.mi_lp_last_error(self.h).decode())
        return r

    # benchmark slicing
    def begin(self, pause_at):
        self._push_params()
        self._check(self._L.mi_lp_begin(self.h, int(pause_at)), "mi_lp_begin")

    def run_until(self, pause_at):
        fin = ctypes.c_int32()
        it = ctypes.c_int64()
        self._check(self._L.mi_lp_run_until(self.h, int(pause_at), ctypes.byref(fin),
                                            ctypes.byref(it)), "mi_lp_run_until")
        return bool(fin.value), int(it.value)

    def stop(self):
        self._check(self._L.mi_lp_stop(self.h), "mi_lp_stop")

    def finish(self):
        r = abi.MiLpResult()
        self._L.mi_lp_finish(self.h, ctypes.byref(r))
        return r

    def kernel_stats(self):
        s = abi.MiLpKernelStats()
        self._L.mi_lp_get_kernel_stats(self.h, ctypes.byref(s))
        return {name: dict(launches=s.launches[i], bytes=s.algorithmic_bytes[i],
                           device_ms=s.device_ms[i], call_ms=s.call_ms[i])
                for i, name in enumerate(abi.KERNEL_NAMES)}

    def set_exchange(self, rank, world, allgather):
        """Cross-process column split (mi_lp_set_exchange): `allgather(data:
        bytes, sizes: list[int]) -> bytes` returns every rank's bytes in rank
        order. Call before load()."""
        self._exchange_cb = allgather_callback(world, allgather)  # kept alive with the handle
        self._check(self._L.mi_lp_set_exchange(self.h, int(rank), int(world), None,
                                               self._exchange_cb), "mi_lp_set_exchange")

    def set_exchange_native(self, rank, world, exchange):
        """Cross-process split with a C++ exchange (ShmExchange): the engine
        calls mi_exchange_allgather directly. Call before load()."""
        ctx, fn = exchange.function()
        self._exchange_keep = (exchange, fn)
        self._check(self._L.mi_lp_set_exchange(self.h, int(rank), int(world), ctx, fn),
                    "mi_lp_set_exchange")

    def record_iteration_times(self, on=True):
        self._check(self._L.mi_lp_record_iteration_times(self.h, int(on)),
                    "mi_lp_record_iteration_times")

    def iteration_times(self):
        """Seconds since Solve() started at the end of every iteration."""
        n = self._L.mi_lp_get_iteration_times(self.h, None, 0)
        if n < 0:
            raise RuntimeError(f"mi_lp_get_iteration_times failed ({-n})")
        out = np.zeros(n)
        self._L.mi_lp_get_iteration_times(self.h, _p(out), n)
        return out

    def run_counters(self):
        c = abi.MiLpRunCounters()
        self._check(self._L.mi_lp_get_run_counters(self.h, ctypes.byref(c)),
                    "mi_lp_get_run_counters")
        return {"factorizations": int(c.factorizations),
                "factorization_seconds": float(c.factorization_seconds),
                "iterations": int(c.iterations), "u_levels": int(c.u_levels),
                "u_outputs": int(c.u_outputs), "u_entries": int(c.u_entries),
                "sdual_segments": int(c.sdual_segments),
                "sdual_iterations": int(c.sdual_iterations)}

    def reset_kernel_stats(self):
        self._L.mi_lp_reset_kernel_stats(self.h)

    def set_kernel_timing(self, on=True, kernels=None):
        """HIP-event timing of the kernel ids in `kernels` (names of
        abi.KERNEL_NAMES; None: all) while on."""
        if kernels is None:
            self._L.mi_lp_set_kernel_timing(self.h, int(on))
            return
        mask = 0
        for k in kernels:
            mask |= 1 << abi.KERNEL_NAMES.index(k)
        self._L.mi_lp_set_kernel_timing_ids(self.h, mask if on else 0)

    def _get(self, fn, n, dtype):
        out = np.zeros(n, dtype=dtype)
        self._check(getattr(self._L, fn)(self.h, _p(out)), fn)
        return out

    def primal(self):
        return self._get("mi_lp_get_primal", self.lp.n, np.float64)

    def reduced_costs(self):
        return self._get("mi_lp_get_reduced_costs", self.lp.n, np.float64)

    def duals(self):
        return self._get("mi_lp_get_duals", self.lp.m, np.float64)

    def activities(self):
        return self._get("mi_lp_get_activities", self.lp.m, np.float64)

    def basis(self):
        return self._get("mi_lp_get_basis", self.lp.m, np.int32)

    def state(self):
        return self._get("mi_lp_get_state", self.lp.n + self.lp.m, np.int8)

    def statuses(self):
        var = np.zeros(self.lp.n, np.int8)
        cons = np.zeros(self.lp.m, np.int8)
        self._check(self._L.mi_lp_get_statuses(self.h, _p(var), _p(cons)),
                    "mi_lp_get_statuses")
        return var, cons

    def primal_ray(self):
        return self._get("mi_lp_get_primal_ray", self.lp.n + self.lp.m, np.float64)

    def dual_ray(self):
        return self._get("mi_lp_get_dual_ray", self.lp.m, np.float64)

    def _call(self, name, *args):
        self._check(getattr(self._L, "mi_lp_" + name)(self.h, *args), "mi_lp_" + name)

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


def batch_solve(handles, num_threads=4, progress=None, progress_s=15.0):
    """Solves already-loaded handles concurrently (mi_lp_batch_solve).

    progress: optional callable(done_indices, elapsed_s), called every
    progress_s seconds while the batch runs and once at the end with the
    indices whose results have landed (a finished solve writes its positive
    solve_seconds or an error code; the entry is zeroed when it starts)."""
    L = lib()
    for h in handles:
        h._push_params()
    arr = (ctypes.c_void_p * len(handles))(*[h.h.value for h in handles])
    res = (abi.MiLpResult * len(handles))()
    if progress is None:
        L.mi_lp_batch_solve(arr, len(handles), num_threads, res)
        return list(res)
    import threading
    import time
    t0 = time.perf_counter()
    th = threading.Thread(target=L.mi_lp_batch_solve,
                          args=(arr, len(handles), num_threads, res), daemon=True)
    th.start()
    while th.is_alive():
        th.join(progress_s)
        progress([i for i, r in enumerate(res) if r.solve_seconds > 0 or r.error_code != 0],
                 time.perf_counter() - t0)
    return list(res)


def batch_solve_gpus(handles, num_gpus, threads_per_gpu=4):
    """Loaded handles on devices [0, num_gpus) solved concurrently, one thread
    pool per device (mi_lp_batch_solve_gpus)."""
    L = lib()
    for h in handles:
        h._push_params()
    arr = (ctypes.c_void_p * len(handles))(*[h.h.value for h in handles])
    res = (abi.MiLpResult * len(handles))()
    rc = L.mi_lp_batch_solve_gpus(arr, len(handles), num_gpus, threads_per_gpu, res)
    if rc != 0:
        raise RuntimeError(f"mi_lp_batch_solve_gpus failed ({rc})")
    return list(res)


def batch_solve_bounds(workers, lbs, ubs, warm_state=None):
    """Children of one search node: LP i = the workers' loaded LP with
    variable bounds lbs[i], ubs[i], warm-started from warm_state
    (mi_lp_batch_solve_bounds). Returns the list of MiLpResult."""
    L = lib()
    for w in workers:
        w._push_params()
    if not workers:
        raise ValueError("batch_solve_bounds needs at least one worker")
    lp = workers[0].lp
    if lp is None or any(w.lp is None or (w.lp.m, w.lp.n) != (lp.m, lp.n) for w in workers):
        raise ValueError("every worker must have the same LP shape loaded")
    lbs = np.ascontiguousarray(lbs, dtype=np.float64)
    ubs = np.ascontiguousarray(ubs, dtype=np.float64)
    if lbs.ndim != 2 or lbs.shape[1] != lp.n:
        raise ValueError(f"lbs must be (count, {lp.n}), got {lbs.shape}")
    if ubs.shape != lbs.shape:
        raise ValueError(f"ubs shape {ubs.shape} != lbs shape {lbs.shape}")
    if warm_state is not None and len(warm_state) != lp.n + lp.m:
        raise ValueError(f"warm_state must have n+m={lp.n + lp.m} entries, "
                         f"got {len(warm_state)}")
    count = lbs.shape[0]
    arr = (ctypes.c_void_p * len(workers))(*[w.h.value for w in workers])
    res = (abi.MiLpResult * count)()
    ws = None if warm_state is None else np.ascontiguousarray(warm_state, dtype=np.int8)
    rc = L.mi_lp_batch_solve_bounds(arr, len(workers), count, _p(lbs), _p(ubs),
                                    None if ws is None else _p(ws),
                                    0 if ws is None else len(ws), res)
    if rc != 0:
        raise RuntimeError(f"mi_lp_batch_solve_bounds failed ({rc})")
    return list(res)


def scale_lp(lp, solver_params=None):
    """ScalingPreprocessor::Run (mi_lp_scale, host only): returns the scaled
    copy of `lp` plus row/column unscaling factors and the cost/bound divisors."""
    from . import lp as lpmod
    L = lib()
    sp = solver_params or abi.default_solver_params()
    cs = np.ascontiguousarray(lp.col_starts, np.int64)
    ri = np.ascontiguousarray(lp.row_idx, np.int32)
    arrs = [np.array(a, np.float64) for a in (lp.vals, lp.col_lb, lp.col_ub, lp.row_lb,
                                              lp.row_ub, lp.obj)]
    off = ctypes.c_double(lp.obj_offset)
    sc = ctypes.c_double(lp.obj_scale)
    rs = np.zeros(lp.m)
    cl = np.zeros(lp.n)
    cf = ctypes.c_double()
    bf = ctypes.c_double()
    rc = L.mi_lp_scale(ctypes.byref(sp), lp.m, lp.n, _p(cs), _p(ri), *[_p(a) for a in arrs],
                       ctypes.byref(off), ctypes.byref(sc), _p(rs), _p(cl), ctypes.byref(cf),
                       ctypes.byref(bf))
    if rc != 0:
        raise ValueError(f"mi_lp_scale failed with {rc}")
    v, clb, cub, rlb, rub, ob = arrs
    out = lpmod.LinearProgram(lp.m, lp.n, cs, ri, v, clb, cub, rlb, rub, ob, off.value,
                              sc.value, lp.maximize, lp.name)
    return out, {"row_scale": rs, "col_scale": cl, "cost_factor": cf.value,
                 "bound_factor": bf.value}


def _lp_arrays(lp):
    return [np.ascontiguousarray(x, dtype=t) for x, t in (
        (lp.col_starts, np.int64), (lp.row_idx, np.int32), (lp.vals, np.float64),
        (lp.col_lb, np.float64), (lp.col_ub, np.float64), (lp.row_lb, np.float64),
        (lp.row_ub, np.float64), (lp.obj, np.float64))]


class Presolve:
    """Glop's MainLpPreprocessor passes and their postsolve (mi_presolve_*,
    host only): run(lp) -> Glop's status after presolve; presolved() -> the
    reduced LinearProgram; recover(...) -> the solution of the original LP."""

    def __init__(self, solver_params=None):
        self._L = lib()
        self.sp = solver_params or abi.default_solver_params(use_preprocessing=1)
        self.h = ctypes.c_void_p(self._L.mi_presolve_create())
        if not self.h:
            raise MemoryError("mi_presolve_create")

    def __del__(self):
        if getattr(self, "h", None):
            self._L.mi_presolve_destroy(self.h)
            self.h = None

    def run(self, lp):
        self.lp = lp
        keep = _lp_arrays(lp)
        st = ctypes.c_int32()
        rc = self._L.mi_presolve_run(self.h, ctypes.byref(self.sp), lp.m, lp.n,
                                     *[_p(a) for a in keep], lp.obj_offset, lp.obj_scale,
                                     int(lp.maximize), ctypes.byref(st))
        if rc != 0:
            raise RuntimeError(f"mi_presolve_run failed ({rc})")
        return st.value

    def passes(self):
        return [self._L.mi_presolve_pass_name(self.h, i).decode()
                for i in range(self._L.mi_presolve_num_passes(self.h))]

    def presolved(self):
        from . import lp as lpmod
        m, n, mx = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        nnz = ctypes.c_int64()
        self._L.mi_presolve_dims(self.h, ctypes.byref(m), ctypes.byref(n), ctypes.byref(nnz),
                                 ctypes.byref(mx))
        m, n, nnz = m.value, n.value, nnz.value
        cs = np.zeros(n + 1, np.int64)
        ri = np.zeros(nnz, np.int32)
        arrs = [np.zeros(k) for k in (nnz, n, n, m, m, n)]
        off, sc = ctypes.c_double(), ctypes.c_double()
        self._L.mi_presolve_get(self.h, _p(cs), _p(ri), *[_p(a) for a in arrs],
                                ctypes.byref(off), ctypes.byref(sc))
        v, clb, cub, rlb, rub, ob = arrs
        return lpmod.LinearProgram(m, n, cs, ri, v, clb, cub, rlb, rub, ob, off.value,
                                   sc.value, bool(mx.value), "presolved")

    def recover(self, status, primal, duals, vstat, cstat):
        p = np.ascontiguousarray(primal, np.float64)
        d = np.ascontiguousarray(duals, np.float64)
        vs = np.ascontiguousarray(vstat, np.int8)
        cst = np.ascontiguousarray(cstat, np.int8)
        n0, m0 = self.lp.n, self.lp.m
        out = {"x": np.zeros(n0), "y": np.zeros(m0), "vstat": np.zeros(n0, np.int8),
               "cstat": np.zeros(m0, np.int8)}
        st = ctypes.c_int32(status)
        rc = self._L.mi_presolve_recover(self.h, ctypes.byref(st), _p(p), _p(d), _p(vs), _p(cst),
                                         *[_p(out[k]) for k in ("x", "y", "vstat", "cstat")])
        if rc != 0:
            raise RuntimeError(f"mi_presolve_recover failed ({rc})")
        return st.value, out


def solve_lp_with(lp, simplex, solver_params=None):
    """mi_lp_solver_solve_with: Glop's LPSolver flow (presolve, scaling, the
    caller's simplex, postsolve, LoadAndVerifySolution) with `simplex(inner_lp)`
    returning (mi_lp_result, primal, duals, vstat, cstat) for the presolved,
    scaled LP. Returns (result, dict of the original LP's solution arrays)."""
    from . import lp as lpmod
    L = lib()
    sp = solver_params or abi.default_solver_params()
    keep = _lp_arrays(lp)
    errors = []

    def cb(user, m, n, cs, ri, v, clb, cub, rlb, rub, ob, off, sc, mx, out, x, y, vs, cst):
        try:
            nnz = ctypes.cast(cs, ctypes.POINTER(ctypes.c_int64))[n] if n >= 0 else 0

            def arr(ptr, k, t):
                if k == 0:
                    return np.zeros(0, t)
                c = {np.float64: ctypes.c_double, np.int64: ctypes.c_int64,
                     np.int32: ctypes.c_int32}[t]
                return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(c)), (k,)).copy()
            inner = lpmod.LinearProgram(
                m, n, arr(cs, n + 1, np.int64), arr(ri, nnz, np.int32), arr(v, nnz, np.float64),
                arr(clb, n, np.float64), arr(cub, n, np.float64), arr(rlb, m, np.float64),
                arr(rub, m, np.float64), arr(ob, n, np.float64), off, sc, bool(mx), "inner")
            r, px, dy, pvs, pcs = simplex(inner)
            ctypes.memmove(out, ctypes.byref(r), ctypes.sizeof(abi.MiLpResult))
            for ptr, a, t in ((x, px, np.float64), (y, dy, np.float64), (vs, pvs, np.int8),
                              (cst, pcs, np.int8)):
                a = np.ascontiguousarray(a, t)
                if a.size:
                    ctypes.memmove(ptr, a.ctypes.data, a.nbytes)
            return 0
        except Exception as exc:  # noqa: BLE001 (reported after the call)
            errors.append(exc)
            return 102

    fn = SIMPLEX_FN(cb)
    out = {"x": np.zeros(lp.n), "y": np.zeros(lp.m), "rc": np.zeros(lp.n),
           "act": np.zeros(lp.m), "vstat": np.zeros(lp.n, np.int8),
           "cstat": np.zeros(lp.m, np.int8)}
    r = abi.MiLpResult()
    rc = L.mi_lp_solver_solve_with(fn, None, ctypes.byref(sp), lp.m, lp.n,
                                   *[_p(a) for a in keep], lp.obj_offset, lp.obj_scale,
                                   int(lp.maximize), ctypes.byref(r),
                                   *[_p(out[k]) for k in ("x", "y", "rc", "act", "vstat",
                                                          "cstat")])
    if errors:
        raise errors[0]
    if rc != 0:
        raise RuntimeError(f"mi_lp_solver_solve_with failed ({rc})")
    return r, out
