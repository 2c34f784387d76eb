"""LPSolver layer: Glop's scaling preprocessor, the
engine solve on the scaled LP and the solution recovery
(or-tools_amd/csrc/engine/lp_solver.cc, C ABI mi_lp_scale / mi_lp_solver_solve).

Checker: oracle/oracle_scaling.py, a numpy restatement of
lp_data/matrix_scaler.cc, lp_data.cc:1144-1258, preprocessor.cc:3855-3912 and
lp_solver.cc:334-367, 540-579, 866-896. CPU tests: the scaled LP and the
scale factors are bit-equal to the restatement (no device needed). GPU
tests: the engine on the scaled LP equals the oracle simplex on the
restatement's scaled LP (pivots, statuses), and the recovered solution of
the original LP equals the restatement's recovery bit for bit; the
known-answer LPs (tests/kat_lps.py, the reference's own test values) reach
their stated objectives through this path."""
import os
import sys

import numpy as np
import pytest

from mi_glop import abi, engine
from mi_glop.lp import LinearProgram

import kat_lps
import lp_gen
import oracle_lib

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "oracle"))
import oracle_scaling  # noqa: E402


def _wide_range_lp(seed, m=40, n=90):
    """Badly scaled LP: rows and columns multiplied by powers of ten, so the
    geometric passes iterate and the cost/bound divisors are not 1."""
    lp = lp_gen.random_sparse_lp(m, n, 0.08, seed)
    rng = np.random.default_rng(seed)
    rs = 10.0 ** rng.integers(-4, 5, m)
    cs = 10.0 ** rng.integers(-3, 4, n)
    vals = lp.vals.copy()
    for c in range(n):
        sl = slice(lp.col_starts[c], lp.col_starts[c + 1])
        vals[sl] = vals[sl] * rs[lp.row_idx[sl]] * cs[c]
    return LinearProgram(m, n, lp.col_starts, lp.row_idx, vals, lp.col_lb / cs,
                         lp.col_ub / cs, lp.row_lb * rs, lp.row_ub * rs,
                         lp.obj * cs * 1e3, 2.5, 1.0, lp.maximize, "wide_range")


def _cases():
    cases = [(f.__name__, f) for f in kat_lps.ALL]
    cases += [(f"wide_{s}", lambda s=s: (_wide_range_lp(s), None)) for s in (1, 2, 3)]
    cases.append(("sparse", lambda: (lp_gen.random_sparse_lp(60, 200, 0.06, 4), None)))
    return cases


def _assert_scaled_equal(lp, cost_scaling):
    sp = abi.default_solver_params(cost_scaling=cost_scaling)
    got, gf = engine.scale_lp(lp, sp)
    want, wf = oracle_scaling.scale_lp(lp, cost_scaling=cost_scaling)
    np.testing.assert_array_equal(got.vals, want["vals"])
    for k in ("obj", "col_lb", "col_ub", "row_lb", "row_ub"):
        np.testing.assert_array_equal(getattr(got, k), want[k], err_msg=k)
    assert got.obj_offset == want["obj_offset"] and got.obj_scale == want["obj_scale"]
    np.testing.assert_array_equal(gf["row_scale"], wf["row_scale"])
    np.testing.assert_array_equal(gf["col_scale"], wf["col_scale"])
    assert gf["cost_factor"] == wf["cost_factor"]
    assert gf["bound_factor"] == wf["bound_factor"]
    return got, gf


@pytest.mark.parametrize("cost_scaling", [abi.NO_COST_SCALING, abi.CONTAIN_ONE_COST_SCALING,
                                          abi.MEAN_COST_SCALING, abi.MEDIAN_COST_SCALING])
@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_scaling_matches_restatement(case, cost_scaling):
    lp, _ = case[1]()
    got, gf = _assert_scaled_equal(lp, cost_scaling)
    if case[0].startswith("wide"):
        # The scaler did real work: every scaled entry is within [1e-3, 1].
        a = np.abs(got.vals)
        assert a.max() <= 1.0 and a.min() > 1e-3
        assert not np.all(gf["row_scale"] == 1.0)


def test_scaling_off_is_identity():
    lp, _ = kat_lps.test_lp()
    got, gf = engine.scale_lp(lp, abi.default_solver_params(use_scaling=0))
    np.testing.assert_array_equal(got.vals, lp.vals)
    assert gf["cost_factor"] == 1.0 and gf["bound_factor"] == 1.0


def test_scale_rejects_bad_rows():
    lp, _ = kat_lps.tiny_lp()
    bad = LinearProgram(lp.m, lp.n, lp.col_starts, np.full_like(lp.row_idx, lp.m), lp.vals,
                        lp.col_lb, lp.col_ub, lp.row_lb, lp.row_ub, lp.obj)
    with pytest.raises(ValueError):
        engine.scale_lp(bad)


@pytest.mark.parametrize("dual", [0, 1])
@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_lp_solver_flow_cpu(case, dual):
    """mi_lp_solver_solve's flow (mi_lp_solver_solve_with: validity checks,
    presolve off, scaling, simplex, RecoverSolution, IsProblemSolutionConsistent,
    LoadAndVerifySolution's values) with the oracle as its simplex equals the
    numpy restatement bit for bit; test_lp_solver_parity runs the same flow
    with the engine behind it on the GPU."""
    lp, expect = case[1]()
    p = abi.default_params(use_dual_simplex=dual)

    def simplex(inner):
        o = oracle_lib.OracleLp(p)
        o.load(inner)
        r = o.solve()
        v, c = o.statuses()
        return r, o.primal(), o.duals(), v, c

    # Presolve off: the numpy restatement covers the scaling layer only
    # (tests/test_presolve.py and test_validate_presolve_gpu.py cover presolve).
    rg, sol = engine.solve_lp_with(lp, simplex, abi.default_solver_params(use_preprocessing=0))
    arr, fac = oracle_scaling.scale_lp(lp)
    slp = LinearProgram(lp.m, lp.n, lp.col_starts, lp.row_idx, arr["vals"], arr["col_lb"],
                        arr["col_ub"], arr["row_lb"], arr["row_ub"], arr["obj"],
                        arr["obj_offset"], arr["obj_scale"], lp.maximize, lp.name)
    o = oracle_lib.OracleLp(p)
    o.load(slp)
    ro = o.solve()
    assert rg.problem_status == ro.problem_status
    assert rg.iterations == ro.iterations
    if ro.problem_status == abi.INVALID_PROBLEM:
        return
    vs, cs = o.statuses()
    np.testing.assert_array_equal(sol["vstat"], vs)
    np.testing.assert_array_equal(sol["cstat"], cs)
    want = oracle_scaling.recover_and_verify(lp, fac, o.primal(), o.duals(), vs,
                                             ro.problem_status == abi.OPTIMAL)
    for k in ("x", "y", "rc", "act"):
        np.testing.assert_array_equal(sol[k], want[k], err_msg=k)
    if ro.problem_status == abi.OPTIMAL:
        assert rg.objective == want["objective"]


@pytest.mark.gpu
@pytest.mark.parametrize("dual", [0, 1])
@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_lp_solver_parity(case, dual):
    lp, expect = case[1]()
    p = abi.default_params(use_dual_simplex=dual)
    g = engine.LpHandle(p)
    rg, sol = g.solve_lp(lp, abi.default_solver_params(use_preprocessing=0))
    # Oracle: the simplex restatement on the restatement's scaled LP.
    arr, fac = oracle_scaling.scale_lp(lp)
    slp = LinearProgram(lp.m, lp.n, lp.col_starts, lp.row_idx, arr["vals"], arr["col_lb"],
                        arr["col_ub"], arr["row_lb"], arr["row_ub"], arr["obj"],
                        arr["obj_offset"], arr["obj_scale"], lp.maximize, lp.name)
    o = oracle_lib.OracleLp(p)
    o.load(slp)
    ro = o.solve()
    assert rg.problem_status == ro.problem_status
    assert rg.iterations == ro.iterations
    if ro.problem_status == abi.INVALID_PROBLEM:
        return
    vs, cs = o.statuses()
    np.testing.assert_array_equal(sol["vstat"], vs)
    np.testing.assert_array_equal(sol["cstat"], cs)
    want = oracle_scaling.recover_and_verify(lp, fac, o.primal(), o.duals(), vs,
                                             ro.problem_status == abi.OPTIMAL)
    for k in ("x", "y", "rc", "act"):
        np.testing.assert_array_equal(sol[k], want[k], err_msg=k)
    if ro.problem_status == abi.OPTIMAL:
        assert rg.objective == want["objective"]
        if expect is not None and "objective" in expect:
            assert abs(rg.objective - expect["objective"]) <= 1e-6 * max(1.0, abs(
                expect["objective"]))


@pytest.mark.gpu
def test_lp_solver_invalid_problem():
    lp, _ = kat_lps.tiny_lp()
    bad = LinearProgram(lp.m, lp.n, lp.col_starts, lp.row_idx, lp.vals, lp.col_ub + 1.0,
                        lp.col_ub, lp.row_lb, lp.row_ub, lp.obj)
    rg, _ = engine.LpHandle().solve_lp(bad)
    assert rg.problem_status == abi.INVALID_PROBLEM


@pytest.mark.parametrize("imprecise", [1, 0])
def test_load_and_verify_flags_imprecise(imprecise):
    """LoadAndVerifySolution's precision checks (lp_solver.cc:369-472): a
    simplex answer whose basic values miss the rows by 1e-3 is IMPRECISE when
    change_status_to_imprecise is set, OPTIMAL otherwise."""
    lp, _ = kat_lps.test_lp()
    p = abi.default_params(use_dual_simplex=1)

    def simplex(inner):
        o = oracle_lib.OracleLp(p)
        o.load(inner)
        r = o.solve()
        v, c = o.statuses()
        x = o.primal().copy()
        x[v == abi.BASIC] += 1e-3
        return r, x, o.duals(), v, c

    r, _ = engine.solve_lp_with(lp, simplex, abi.default_solver_params(
        change_status_to_imprecise=imprecise, use_preprocessing=0))
    assert r.problem_status == (abi.IMPRECISE if imprecise else abi.OPTIMAL)
