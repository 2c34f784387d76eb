"""LpScalingHelper (mi_glop.scaling; lp_data/lp_data_utils.cc:76-182) and the
CP-SAT LP constraint on a scaled LP (linear_programming_constraint.cc:417,
:683-686, :699-707, :849, :2367-2408). CPU only: the scaling runs in the
engine library's host-only mi_lp_scale, the solves on the oracle."""
import math

import numpy as np

from mi_glop import abi, cpsat
from mi_glop.scaling import LpScalingHelper

import jobshop
import lp_gen
import oracle_lib


def _solve(lp, params):
    o = oracle_lib.OracleLp(params)
    o.load(lp)
    r = o.solve()
    return o, r


def test_factors_follow_the_reference_formulas():
    lp = lp_gen.random_sparse_lp(60, 150, 0.06, 11)
    h = LpScalingHelper()
    scaled = h.scale(lp, abi.default_solver_params(cost_scaling=abi.MEAN_COST_SCALING))
    assert h.col_unscale.shape == (lp.n,) and h.row_unscale.shape == (lp.m,)
    assert h.bound_scaling_factor > 0 and h.objective_scaling_factor > 0
    # Bounds of the scaled LP are the original ones times VariableScalingFactor
    # (Scale divides by the column scale, ScaleBounds by the bound divisor).
    for c in range(lp.n):
        f = h.variable_scaling_factor(c)
        assert f == h.col_unscale[c] * h.bound_scaling_factor
        for a, b in ((lp.col_lb[c], scaled.col_lb[c]), (lp.col_ub[c], scaled.col_ub[c])):
            if math.isfinite(a):
                assert math.isclose(a * f, b, rel_tol=1e-14, abs_tol=1e-300)
    # Scale and unscale are inverse up to one rounding each.
    for c in range(0, lp.n, 7):
        for v in (0.0, 1.5, -3.25e4):
            assert math.isclose(h.unscale_variable_value(c, h.scale_variable_value(c, v)), v,
                                rel_tol=4e-16)
            assert math.isclose(h.unscale_reduced_cost(c, h.scale_reduced_cost(c, v)), v,
                                rel_tol=4e-16)
    for r in range(0, lp.m, 5):
        for v in (2.0, -7.5):
            assert math.isclose(h.unscale_dual_value(r, h.scale_dual_value(r, v)), v, rel_tol=4e-16)
            assert math.isclose(h.unscale_constraint_activity(r, h.scale_constraint_activity(r, v)),
                                v, rel_tol=4e-16)
    # The vectorised forms are the scalar ones element-wise.
    x = np.linspace(-3, 5, lp.n)
    assert np.array_equal(h.unscale_variable_values(x),
                          np.array([h.unscale_variable_value(c, x[c]) for c in range(lp.n)]))
    h.clear()
    assert h.variable_scaling_factor(3) == 1.0 and h.unscale_variable_value(3, 2.5) == 2.5


def test_scaled_solve_unscales_to_the_unscaled_solution():
    lp = lp_gen.random_sparse_lp(80, 200, 0.05, 23)
    p = abi.default_params()
    _, r0 = _solve(lp, p)
    o0 = oracle_lib.OracleLp(p)
    o0.load(lp)
    o0.solve()
    h = LpScalingHelper()
    scaled = h.scale(lp)
    o1, r1 = _solve(scaled, p)
    assert r0.problem_status == r1.problem_status == abi.OPTIMAL
    # The scaled LP's objective scaling factor carries the objective back.
    assert math.isclose(r0.objective, r1.objective, rel_tol=1e-9, abs_tol=1e-9)
    x0 = np.asarray(o0.primal())
    x1 = h.unscale_variable_values(o1.primal())
    assert np.allclose(x0, x1, rtol=1e-7, atol=1e-7)
    y0 = np.asarray(o0.duals())
    y1 = h.unscale_dual_values(o1.duals())
    assert np.allclose(y0, y1, rtol=1e-7, atol=1e-7)


def test_scaled_lp_constraint_matches_the_unscaled_one():
    """The LP constraint over the scaled ft06 relaxation reaches the same root
    bound, an LP solution equal up to rounding, and deductions within one
    integer of the unscaled constraint's (the scaled simplex pivots differently
    on ties, so the LP optimum's vertex may differ; the bound may not)."""
    lp, ycols = jobshop.relaxation(jobshop.FT06)
    p = abi.default_params(use_dual_simplex=1)
    plain = cpsat.LpConstraint(lp, ycols, oracle_lib.OracleLp(p))
    scaled = cpsat.LpConstraint(lp, ycols, oracle_lib.OracleLp(p), scaling=True)
    assert scaled.scaler.col_unscale is not None
    t0 = cpsat.IntegerTrail(lp.col_lb, lp.col_ub, obj_ub=60.0)
    t1 = cpsat.IntegerTrail(lp.col_lb, lp.col_ub, obj_ub=60.0)
    assert plain.propagate(t0) and scaled.propagate(t1)
    assert math.isclose(plain.lp_objective, scaled.lp_objective, rel_tol=1e-9)
    assert t0.obj_lb == t1.obj_lb
    # Bounds the simplex sees are the CP bounds times the factors.
    lbs, ubs = scaled.scale_bounds(t1.lb, t1.ub)
    assert np.array_equal(lbs, t1.lb * scaled.factor)
    # Every deduction of the scaled constraint is the reference's formula on
    # the scaled simplex values, unscaled (:2380-2386).
    t2 = cpsat.IntegerTrail(lp.col_lb, lp.col_ub, obj_ub=60.0)
    rc = np.asarray(scaled.h.reduced_costs())
    x = np.asarray(scaled.h.primal())
    delta = 60.0 - scaled.lp_objective
    for col, kind, v in scaled.reduced_cost_deductions(t2, delta, rc, x):
        other = scaled.scaler.unscale_variable_value(
            col, x[col] + (delta / scaled.lp_data.obj_scale) / rc[col])
        if kind == "le":
            assert rc[col] > cpsat.K_LP_EPSILON and v == math.floor(other + cpsat.K_CP_EPSILON)
        else:
            assert rc[col] < -cpsat.K_LP_EPSILON and v == math.ceil(other - cpsat.K_CP_EPSILON)
    # The stored reduced costs are the simplex's, unscaled (:849).
    assert np.array_equal(scaled.reduced_costs, scaled.scaler.unscale_reduced_costs(rc))
