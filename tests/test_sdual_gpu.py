"""The device dual simplex segment on the MI355X (or-tools_amd/csrc/sdual):
phase-II dual iterations run whole on one workgroup, the host engine keeps the
factorizations and the loop's other branches. Every result must equal the
oracle's bit for bit, and the segments must have run on the device."""
import math
import os

import numpy as np
import pytest

from mi_glop import abi, cpsat, engine
import jobshop
import lp_gen
import oracle_lib
import parity_util

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _segments_on(monkeypatch):
    """Segments in every batch call of this file: by default a batch with
    fewer than MILP_SDUAL_MIN_LPS (512) LPs in flight takes the
    batched-launch path (simplex.cc SetBatchMode)."""
    monkeypatch.setenv("MILP_SDUAL", "device")


@pytest.fixture(params=["device", "host"])
def sdual_mode(request, monkeypatch):
    monkeypatch.setenv("MILP_SDUAL", request.param)
    return request.param


@pytest.mark.parametrize("seed", range(4))
def test_sdual_single_lp_parity(seed, sdual_mode):
    m, n = 60 + 50 * seed, 240 + 150 * seed
    lp = lp_gen.random_sparse_lp(m, n, 0.05, 900 + seed, maximize=bool(seed % 2))
    p = abi.default_params(use_dual_simplex=1)
    o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q, 0))
    parity_util.compare(o, ro, g, rg, lp)
    c = g.run_counters()
    assert c["sdual_segments"] > 0 and c["sdual_iterations"] > 0, c
    if sdual_mode == "device":
        assert g.kernel_stats()["sdual"]["launches"] == c["sdual_segments"]


@pytest.mark.parametrize("seed", range(4))
def test_sdual_dual_phase1_parity(seed, sdual_mode, monkeypatch):
    """Glop's dedicated dual phase I (revised_simplex.cc:2198-2388,
    entering_variable.cc:241-355) in segments: LPs whose slack basis is dual
    infeasible on unboxed columns (seed 3 is dual infeasible), from scratch.
    The whole final state equals the oracle's, and the segments ran more
    iterations than with phase I on the host (MILP_SDUAL_PHASE1=0)."""
    m, n = 80 + 60 * seed, 300 + 200 * seed
    lp = lp_gen.dual_phase1_lp(m, n, 910 + seed, unbounded_cols=2 if seed == 3 else 0)
    p = abi.default_params(use_dual_simplex=1)
    counters = []
    for phase1 in ("1", "0"):
        monkeypatch.setenv("MILP_SDUAL_PHASE1", phase1)
        o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q, 0))
        parity_util.compare(o, ro, g, rg, lp)
        counters.append(g.run_counters())
    assert counters[0]["sdual_iterations"] > counters[1]["sdual_iterations"], counters


@pytest.mark.parametrize("kind", ["sparse", "phase1"])
def test_sdual_pfi_parity(kind, sdual_mode):
    """The product-form (eta) updates, use_middle_product_form_update = false
    (basis_representation.cc:25-176), in segments on one workgroup: the
    whole final state equals the oracle's."""
    if kind == "sparse":
        lp = lp_gen.random_sparse_lp(160, 600, 0.04, 731)
    else:
        lp = lp_gen.dual_phase1_lp(200, 700, 961)
    p = abi.default_params(use_dual_simplex=1, use_middle_product_form_update=0)
    o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q, 0))
    parity_util.compare(o, ro, g, rg, lp)
    c = g.run_counters()
    assert c["sdual_segments"] > 0 and c["sdual_iterations"] > 0, c


def test_sdual_dual_phase1_batch():
    """Phase-I LPs through the batch API (the pool kernel on the device, 4
    workers): each result equals the oracle solving it alone."""
    lps = [lp_gen.dual_phase1_lp(70 + 30 * k, 260 + 90 * k, 930 + k) for k in range(8)]
    p = abi.default_params(use_dual_simplex=1)
    handles = []
    for lp in lps:
        h = engine.LpHandle(p)
        h.load(lp)
        handles.append(h)
    res = engine.batch_solve(handles, 4)
    for k, (lp, r) in enumerate(zip(lps, res)):
        o = oracle_lib.OracleLp(p)
        o.load(lp)
        ro = o.solve()
        assert (r.error_code, r.problem_status, r.iterations) == \
            (ro.error_code, ro.problem_status, ro.iterations), k
        assert r.objective == ro.objective, (k, r.objective, ro.objective)
    assert sum(h.run_counters()["sdual_iterations"] for h in handles) > 0


def _children(shape, count, seed=3):
    jobs = jobshop.FT06 if shape == (6, 6) else jobshop.random_instance(*shape, seed)
    lp, ycols = jobshop.relaxation(jobs)
    root = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=1))
    root.load(lp)
    rr = root.solve()
    state, x = root.state(), root.primal()
    node = cpsat.IntegerTrail(lp.col_lb, lp.col_ub,
                              obj_lb=math.ceil(rr.objective - cpsat.K_CP_EPSILON))
    cols = cpsat.fractional_columns(x, ycols, limit=count // 2)
    lbs, ubs = cpsat.branch_lps(node, x, cols)
    return lp, state, lbs, ubs


@pytest.mark.parametrize("shape", [(6, 6), (15, 10)])
def test_sdual_children_parity(shape, sdual_mode):
    """Config-4 children through the batch API (4 workers, fibers) with the
    segments on; each child equals the oracle solving it alone."""
    lp, state, lbs, ubs = _children(shape, 24)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    workers = [engine.LpHandle(p) for _ in range(4)]
    for w in workers:
        w.load(lp)
    res = engine.batch_solve_bounds(workers, lbs, ubs, state)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    for i, r in enumerate(res):
        o.set_variable_bounds(lbs[i], ubs[i])
        o.load_basis_state(state)
        ro = o.solve()
        assert (r.error_code, r.problem_status, r.iterations) == \
            (ro.error_code, ro.problem_status, ro.iterations), i
        assert r.objective == ro.objective, (i, r.objective, ro.objective)
    segs = sum(w.run_counters()["sdual_segments"] for w in workers)
    assert segs > 0


@pytest.mark.parametrize("shape", [(6, 6), (15, 10)])
def test_sdual_children_shared_caches(shape, monkeypatch):
    """A node's children with and without the shared first factorization and
    dual edge norms (MILP_BATCH_SHARED_LU, MILP_BATCH_SHARED_NORMS): every
    child equals the oracle solving it alone. The deterministic time is
    cumulative per handle (as Glop's RevisedSimplex keeps it), so it is
    compared on one worker, whose children run in order like the oracle's
    reused handle: equal to the oracle's with the caches on or off (a cache
    hit replays the bumps)."""
    monkeypatch.setenv("MILP_SDUAL", "device")
    lp, state, lbs, ubs = _children(shape, 24)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    ref = []
    for i in range(len(lbs)):
        o.set_variable_bounds(lbs[i], ubs[i])
        o.load_basis_state(state)
        ref.append(o.solve())
    for shared in ("0", "1"):
        monkeypatch.setenv("MILP_BATCH_SHARED_LU", shared)
        monkeypatch.setenv("MILP_BATCH_SHARED_NORMS", shared)
        for nw in (8, 1):
            workers = [engine.LpHandle(p) for _ in range(nw)]
            for w in workers:
                w.load(lp)
            res = engine.batch_solve_bounds(workers, lbs, ubs, state)
            for i, (r, ro) in enumerate(zip(res, ref)):
                assert (r.error_code, r.problem_status, r.iterations) == \
                    (ro.error_code, ro.problem_status, ro.iterations), (shared, nw, i)
                assert r.objective == ro.objective, (shared, nw, i, r.objective, ro.objective)
                if nw == 1:
                    assert r.deterministic_time == ro.deterministic_time, (shared, i)


def test_sdual_child_full_state(sdual_mode):
    """One child on one handle: the whole final state, not just the result."""
    lp, state, lbs, ubs = _children((10, 5), 6, seed=5)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    for i in range(len(lbs)):
        g = engine.LpHandle(p, 0)
        g.load(lp)
        g.set_variable_bounds(lbs[i], ubs[i])
        g.load_basis_state(state)
        rg = g.solve()
        o = oracle_lib.OracleLp(p)
        o.load(lp)
        o.set_variable_bounds(lbs[i], ubs[i])
        o.load_basis_state(state)
        ro = o.solve()
        parity_util.compare(o, ro, g, rg, lp)


def test_sdual_pool_at_bench_scale():
    """The pool at the benchmark's scale (bench.py's config-4 section runs
    1 024 handles): 512 children of the 15x10 node with 256 LPs in flight,
    each equal to the oracle solving it alone."""
    lp, state, lbs, ubs = _children((15, 10), 512)
    assert len(lbs) >= 256
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    workers = [engine.LpHandle(p) for _ in range(256)]
    for w in workers:
        w.load(lp)
    got = engine.batch_solve_bounds(workers, lbs, ubs, state)
    ows = [oracle_lib.OracleLp(p) for _ in range(8)]
    for w in ows:
        w.load(lp)
    ref = oracle_lib.batch_solve_bounds(ows, lbs, ubs, state)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert (a.error_code, a.problem_status, a.iterations) == \
            (b.error_code, b.problem_status, b.iterations), i
        assert a.objective == b.objective, (i, a.objective, b.objective)
    assert sum(w.run_counters()["sdual_segments"] for w in workers) > 0


_WRAP = r"""
import sys
sys.path[:0] = ["tests", "or-tools_amd"]
from mi_glop import abi, engine
import oracle_lib
import test_sdual_gpu as t
lp, state, lbs, ubs = t._children((10, 5), 40, seed=11)
p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
workers = [engine.LpHandle(p) for _ in range(16)]
for w in workers:
    w.load(lp)
ows = [oracle_lib.OracleLp(p) for _ in range(4)]
for w in ows:
    w.load(lp)
ref = oracle_lib.batch_solve_bounds(ows, lbs, ubs, state)
for call in range(3):
    got = engine.batch_solve_bounds(workers, lbs, ubs, state)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert (a.error_code, a.problem_status, a.iterations, a.objective) == \
            (b.error_code, b.problem_status, b.iterations, b.objective), (call, i)
segs = sum(w.run_counters()["sdual_segments"] for w in workers)
print("OK segments", segs)
"""


def test_sdual_pool_queue_wraparound():
    """More segments than the queue's slots through the pool: the rings are
    cut to 8 slots (MILP_SDUAL_QUEUE_CAP, read when the pool is created, so
    in a fresh process), three batch calls back to back (the last batch call
    stops the grid, the next relaunches it from the first uncopied entry);
    every child still equals the oracle."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MILP_SDUAL_QUEUE_CAP="8", MILP_SDUAL="device")
    r = subprocess.run([sys.executable, "-c", _WRAP], cwd=repo, env=env, timeout=240,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    segs = int(r.stdout.split("OK segments")[1].split()[0])
    assert segs > 3 * 8, segs
