"""Glop's presolve (MainLpPreprocessor, glop/preprocessor.cc:76-147) and the
LPSolver flow around it (lp_solver.cc:150-261), host code in
or-tools_amd/csrc/engine/presolve.cc + lp_solver.cc, C ABI mi_presolve_* and
mi_lp_solver_solve_with.

CPU tests. The simplex behind the flow is the oracle (tests/oracle_lib.py)
passed as the caller-supplied simplex of mi_lp_solver_solve_with; the engine
is the same simplex bit for bit (tests/test_parity_gpu.py), so the GPU path
(mi_lp_solver_solve) differs only in that callback.

Parity of the presolved LP itself is unpinned: the reference's presolve is
C++ that needs absl/protobuf to build (unbuildable here) and the reference
holds no presolve fixtures. The checks are the size-independent properties
of a correct presolve + postsolve on every LP of tests/lp_gen.presolve_lp
(which makes each of the 14 passes fire) and of the known-answer LPs:
- the same status and optimal objective as the unpresolved flow (1e-9
  relative; measured 8.7e-14),
- a postsolved solution that passes LPSolver's own IsProblemSolutionConsistent
  (lp_solver.cc:679-790: statuses at their bounds, exactly m basic), else the
  flow reports ABNORMAL,
- primal and dual feasibility of the postsolved solution on the original LP,
plus hand-derived exact reductions for the simple passes."""
import numpy as np
import pytest

from mi_glop import abi, engine
from mi_glop.lp import LinearProgram

import kat_lps
import lp_gen
import oracle_lib

INF = np.inf
ALL_PASSES = {"ShiftVariableBounds", "FixedVariable", "Singleton",
              "ForcingAndImpliedFreeConstraint", "FreeConstraint", "ImpliedFree",
              "UnconstrainedVariable", "DoubletonFreeColumn", "DoubletonEqualityRow",
              "EmptyColumn", "EmptyConstraint", "ProportionalColumn", "ProportionalRow",
              "Dualizer", "SingletonColumnSign"}


def oracle_simplex(params):
    def run(inner):
        o = oracle_lib.OracleLp(params)
        o.load(inner)
        r = o.solve()
        v, c = o.statuses()
        return r, o.primal(), o.duals(), v, c
    return run


def _solve(lp, presolve, dual=1, **kw):
    p = abi.default_params(use_dual_simplex=dual)
    sp = abi.default_solver_params(use_preprocessing=int(presolve), **kw)
    return engine.solve_lp_with(lp, oracle_simplex(p), sp)


def _assert_feasible(lp, sol, tol=1e-9):
    x, act = sol["x"], sol["act"]
    assert np.all(x >= lp.col_lb - tol) and np.all(x <= lp.col_ub + tol)
    scale = lambda b: np.maximum(1.0, np.abs(np.where(np.isfinite(b), b, 0.0)))  # noqa: E731
    assert np.all(act >= lp.row_lb - tol * scale(lp.row_lb))
    assert np.all(act <= lp.row_ub + tol * scale(lp.row_ub))
    sign = -1.0 if lp.maximize else 1.0
    rc = sign * sol["rc"]
    above_lb = x > lp.col_lb + tol
    below_ub = x < lp.col_ub - tol
    assert np.all(rc[above_lb] <= tol) and np.all(rc[below_ub] >= -tol)
    # Complementary slackness on the rows (minimization sense): a row strictly
    # above its lower bound has dual <= 0, strictly below its upper bound >= 0.
    y = sign * sol["y"]
    assert np.all(y[act > lp.row_lb + tol * scale(lp.row_lb)] <= tol)
    assert np.all(y[act < lp.row_ub - tol * scale(lp.row_ub)] >= -tol)


@pytest.mark.parametrize("tall", [False, True], ids=["wide", "tall"])
@pytest.mark.parametrize("seed", range(12))
def test_presolve_matches_unpresolved(seed, tall):
    lp = lp_gen.presolve_lp(40 + 3 * seed, 90 + 5 * seed, 500 + seed,
                            maximize=bool(seed % 2), tall=tall)
    r0, s0 = _solve(lp, False)
    r1, s1 = _solve(lp, True)
    assert r0.problem_status == abi.OPTIMAL
    assert r1.problem_status == abi.OPTIMAL, "postsolved solution inconsistent (ABNORMAL)"
    assert abs(r1.objective - r0.objective) <= 1e-9 * max(1.0, abs(r0.objective))
    _assert_feasible(lp, s1)
    ps = engine.Presolve()
    assert ps.run(lp) == abi.INIT
    red = ps.presolved()
    if tall:
        # The dual of the reduced LP: one row per remaining primal column.
        assert "Dualizer" in ps.passes() and red.maximize and red.m < lp.n
    else:
        assert red.m < lp.m and red.n < lp.n


def test_presolve_every_pass_fires():
    """Every pass changes some LP, except EmptyColumnPreprocessor: in Glop's
    order UnconstrainedVariablePreprocessor (preprocessor.cc:1841-2083) has
    already removed every empty column (its reduced-cost bounds are the cost
    alone) or reported INFEASIBLE_OR_UNBOUNDED before EmptyColumn runs."""
    seen = set()
    for seed in range(16):
        for tall in (False, True):
            ps = engine.Presolve()
            ps.run(lp_gen.presolve_lp(40 + seed, 90 + 2 * seed, 700 + seed, tall=tall))
            seen.update(ps.passes())
    assert seen == ALL_PASSES - {"EmptyColumn"}, ALL_PASSES - seen


@pytest.mark.parametrize("f", kat_lps.ALL, ids=lambda f: f.__name__)
def test_presolve_known_answers(f):
    lp, expect = f()
    r, sol = _solve(lp, True)
    if "status" in expect:
        assert r.problem_status == expect["status"]
    if "status_in" in expect:
        # Presolve may decide the class first (INFEASIBLE_OR_UNBOUNDED,
        # preprocessor.cc:427, 584, 1962, 2756).
        allowed = {getattr(abi, s) for s in expect["status_in"]} | {abi.INFEASIBLE_OR_UNBOUNDED}
        assert r.problem_status in allowed
    if "objective" in expect and r.problem_status == abi.OPTIMAL:
        assert abs(r.objective - expect["objective"]) <= 1e-6 * max(1.0, abs(expect["objective"]))
        _assert_feasible(lp, sol, 1e-7)


@pytest.mark.parametrize("dual", [0, 1])
@pytest.mark.parametrize("seed", range(6))
def test_presolve_suite_lps(seed, dual):
    lp = lp_gen.random_sparse_lp(45 + 10 * seed, 130 + 20 * seed, 0.05, 900 + seed,
                                 maximize=bool(seed % 2))
    r0, _ = _solve(lp, False, dual)
    r1, s1 = _solve(lp, True, dual)
    assert (r0.problem_status, r1.problem_status) == (abi.OPTIMAL, abi.OPTIMAL)
    assert abs(r1.objective - r0.objective) <= 1e-9 * max(1.0, abs(r0.objective))
    _assert_feasible(lp, s1)


def _lp(rows, col_lb, col_ub, row_lb, row_ub, obj, maximize=False, offset=0.0):
    a = np.asarray(rows, float).reshape(len(row_lb), len(col_lb))
    return LinearProgram.from_dense(a, col_lb, col_ub, row_lb, row_ub, obj, offset,
                                    maximize=maximize)


def test_fixed_and_empty_reductions():
    """ShiftVariableBoundsPreprocessor (preprocessor.cc:3740-3821) shifts x1 by
    2 and x2 by 1 (row 0 becomes [-5, 4], offset 0.5 + 4 + 1);
    FixedVariablePreprocessor (:1090-1110) removes x1; the empty x2 (cost 1)
    goes to its lower bound in UnconstrainedVariablePreprocessor (:1920-1952);
    EmptyConstraintPreprocessor (:2204-2238) drops row 1. The postsolve puts
    the shifted bounds back (:3823-3849): x = [4, 2, 1], objective 1.5."""
    lp = _lp([[1, 3, 0], [0, 0, 0]], [0, 2, 1], [4, 2, 5], [1, -1], [10, 1], [-1, 2, 1],
             offset=0.5)
    ps = engine.Presolve()
    ps.run(lp)
    passes = ps.passes()
    assert passes[:2] == ["ShiftVariableBounds", "FixedVariable"]
    assert "UnconstrainedVariable" in passes and "EmptyConstraint" in passes
    red = ps.presolved()
    assert red.n <= 1 and red.m <= 1
    r, sol = _solve(lp, True)
    assert r.problem_status == abi.OPTIMAL
    np.testing.assert_array_equal(sol["x"], [4.0, 2.0, 1.0])
    assert r.objective == -4.0 + 4.0 + 1.0 + 0.5
    assert sol["vstat"][1] == abi.FIXED_VALUE and sol["vstat"][2] == abi.AT_LOWER_BOUND


def test_singleton_row_becomes_bounds():
    """SingletonPreprocessor::DeleteSingletonRow (preprocessor.cc:2284-2351):
    2 x0 <= 6 tightens x0 <= 3 and the row goes; the postsolve makes the row
    AT_UPPER_BOUND with dual rc / 2 when x0 ends at the implied bound
    (SingletonRowUndo, :2354-2424)."""
    lp = _lp([[2, 0], [1, 1]], [0, 0], [10, 10], [-INF, -INF], [6, 8], [-3, -1])
    r, sol = _solve(lp, True)
    r0, sol0 = _solve(lp, False)
    assert r.problem_status == abi.OPTIMAL
    assert r.objective == r0.objective == -3 * 3 - 5
    np.testing.assert_array_equal(sol["x"], sol0["x"])
    np.testing.assert_array_equal(sol["y"], sol0["y"])
    assert sol["cstat"][0] == abi.AT_UPPER_BOUND


def test_presolve_detects_infeasible_and_unbounded():
    """EmptyConstraintPreprocessor: an empty row whose range excludes 0 is
    PRIMAL_INFEASIBLE (:2223-2233); EmptyColumnPreprocessor: an empty column
    with a cost towards an infinite bound is INFEASIBLE_OR_UNBOUNDED (:420-429)."""
    infeasible = _lp([[1, 1], [0, 0]], [0, 0], [1, 1], [0, 1], [2, 2], [1, 1])
    ps = engine.Presolve()
    assert ps.run(infeasible) == abi.PRIMAL_INFEASIBLE
    r, _ = _solve(infeasible, True)
    assert r.problem_status == abi.PRIMAL_INFEASIBLE
    unbounded = _lp([[1, 0]], [0, 0], [1, INF], [0], [1], [1, -1])
    ps = engine.Presolve()
    assert ps.run(unbounded) == abi.INFEASIBLE_OR_UNBOUNDED
    r, _ = _solve(unbounded, True)
    assert r.problem_status == abi.INFEASIBLE_OR_UNBOUNDED


def test_use_preprocessing_off_is_identity():
    lp = lp_gen.presolve_lp(40, 90, 3)
    ps = engine.Presolve(abi.default_solver_params(use_preprocessing=0))
    assert ps.run(lp) == abi.INIT and ps.passes() == []
    red = ps.presolved()
    for k in ("col_starts", "row_idx", "vals", "col_lb", "col_ub", "row_lb", "row_ub", "obj"):
        np.testing.assert_array_equal(getattr(red, k), getattr(lp, k), err_msg=k)


def test_presolve_abi_state_rules():
    lp = lp_gen.presolve_lp(30, 60, 11)
    ps = engine.Presolve()
    st = ps.run(lp)
    with pytest.raises(RuntimeError):
        ps.run(lp)  # once per object
    red = ps.presolved()
    r, px, dy, vs, cs = oracle_simplex(abi.default_params(use_dual_simplex=1))(red)
    st2, out = ps.recover(r.problem_status if st == abi.INIT else st, px, dy, vs, cs)
    assert st2 == abi.OPTIMAL and out["x"].shape == (lp.n,) and out["y"].shape == (lp.m,)
    assert int((out["vstat"] == abi.BASIC).sum() + (out["cstat"] == abi.BASIC).sum()) == lp.m
    with pytest.raises(RuntimeError):
        ps.recover(st2, px, dy, vs, cs)  # DestructiveRecoverSolution: once


@pytest.mark.parametrize("seed", range(3))
def test_dualizer_always(seed):
    """solve_dual_problem = ALWAYS_DO (parameters.proto:42-46): the dual is
    solved and mapped back (DualizerPreprocessor::RecoverSolution,
    preprocessor.cc:3607-3714)."""
    lp = lp_gen.presolve_lp(40, 80, 800 + seed, maximize=bool(seed % 2))
    r0, _ = _solve(lp, False)
    r1, s1 = _solve(lp, True, solve_dual_problem=abi.ALWAYS_DO)
    ps = engine.Presolve(abi.default_solver_params(use_preprocessing=1,
                                                   solve_dual_problem=abi.ALWAYS_DO))
    ps.run(lp)
    assert "Dualizer" in ps.passes()
    assert (r0.problem_status, r1.problem_status) == (abi.OPTIMAL, abi.OPTIMAL)
    assert abs(r1.objective - r0.objective) <= 1e-9 * max(1.0, abs(r0.objective))
    _assert_feasible(lp, s1)


_SLACK_OF = {abi.BASIC: abi.BASIC, abi.FIXED_VALUE: abi.FIXED_VALUE,
             abi.AT_LOWER_BOUND: abi.AT_UPPER_BOUND, abi.AT_UPPER_BOUND: abi.AT_LOWER_BOUND,
             abi.FREE: abi.FREE}


@pytest.mark.parametrize("scaling", [0, 1])
@pytest.mark.parametrize("seed", range(8))
def test_postsolved_basis_is_an_optimal_basis(seed, scaling):
    """The postsolved statuses, loaded as a warm start into the simplex on the
    original LP (constraint -> slack status as LPSolver::SetInitialBasis,
    lp_solver.cc:268-299), are a nonsingular, primal and dual feasible basis:
    the simplex stops after 0 iterations at the same objective."""
    for tall in (False, True):
        lp = lp_gen.presolve_lp(40 + seed, 90 + 2 * seed, 1200 + seed,
                                maximize=bool(seed % 2), tall=tall)
        p = abi.default_params(use_dual_simplex=1)
        r, sol = _solve(lp, True, 1, use_scaling=scaling)
        assert r.problem_status == abi.OPTIMAL
        state = np.concatenate([sol["vstat"], [_SLACK_OF[int(c)] for c in sol["cstat"]]])
        o = oracle_lib.OracleLp(p)
        o.load(lp)
        o.load_basis_state(state.astype(np.int8))
        ro = o.solve()
        assert (ro.problem_status, ro.iterations) == (abi.OPTIMAL, 0), (seed, tall)
        assert abs(ro.objective - r.objective) <= 1e-9 * max(1.0, abs(r.objective))


def test_presolve_rejects_invalid_lp():
    """LPSolver checks IsValid before presolve (lp_solver.cc:196-202)."""
    lp = _lp([[1, 1]], [0, 2], [1, 1], [0], [1], [1, 1])  # x1 has lb > ub
    ps = engine.Presolve()
    assert ps.run(lp) == abi.INVALID_PROBLEM and ps.passes() == []
    r, _ = _solve(lp, True)
    assert r.problem_status == abi.INVALID_PROBLEM


@pytest.mark.parametrize("seed", range(4))
def test_presolve_fuzz_statuses(seed):
    """Small LPs of every bound type, most of them infeasible or unbounded:
    with and without presolve the flow agrees (both OPTIMAL with the same
    objective, or both non-optimal with statuses consistent with what the
    primal and dual simplex report unpresolved; never ABNORMAL/IMPRECISE from
    presolve). 5 000 such LPs ran clean while the passes were written."""
    rng = np.random.default_rng(4000 + seed)
    for t in range(250):
        lp = lp_gen.tiny_mixed_lp(rng, 9)
        res = {}
        for dual in (0, 1):
            res[dual] = (_solve(lp, False, dual)[0], _solve(lp, True, dual)[0])
        base = {res[d][0].problem_status for d in (0, 1)}
        for dual in (0, 1):
            r0, r1 = res[dual]
            a, b = r0.problem_status, r1.problem_status
            if a == abi.OPTIMAL or b == abi.OPTIMAL:
                assert a == b == abi.OPTIMAL, (t, dual, a, b)
                assert abs(r0.objective - r1.objective) <= 1e-9 * max(1.0, abs(r0.objective))
                continue
            assert b not in (abi.ABNORMAL, abi.IMPRECISE), (t, dual, a, b)
            if base & {abi.PRIMAL_INFEASIBLE, abi.DUAL_UNBOUNDED}:
                assert b in (abi.PRIMAL_INFEASIBLE, abi.DUAL_INFEASIBLE,
                             abi.INFEASIBLE_OR_UNBOUNDED, abi.DUAL_UNBOUNDED), (t, dual, a, b)
            elif abi.PRIMAL_UNBOUNDED in base:
                assert b in (abi.DUAL_INFEASIBLE, abi.INFEASIBLE_OR_UNBOUNDED,
                             abi.PRIMAL_UNBOUNDED), (t, dual, a, b)
