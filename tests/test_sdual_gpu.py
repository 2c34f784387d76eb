"""The device dual simplex segment on the MI355X (or-tools_amd/csrc/sdual):
phase-II dual iterations run whole on one workgroup, the host engine keeps the
factorizations and the loop's other branches. Every result must equal the
oracle's bit for bit, and the segments must have run on the device."""
import math

import numpy as np
import pytest

from mi_glop import abi, cpsat, engine
import jobshop
import lp_gen
import oracle_lib
import parity_util

pytestmark = pytest.mark.gpu


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
