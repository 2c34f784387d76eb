"""CP-SAT LP call-out semantics (mi_glop.cpsat; sat/linear_programming_constraint.cc
SolveLp :709-760, AnalyzeLp :762-860, ReducedCostStrengtheningDeductions
:2367-2408, BranchOnVar :485-584, SolveLpForBranching :443-464).

CPU: the driver runs on the oracle (the CPU restatement stands in for the
engine: the driver only needs the handle surface); its BranchOnVar folding
is checked case by case, and the batched node (every branch LP solved from
the node's state in one batch call) is checked to solve exactly the LPs the
sequential SolveLpForBranching solves. GPU: the engine's batch over a node's
branch LPs equals the oracle's, bit for bit, and folds to the same node."""
import math

import numpy as np
import pytest

from mi_glop import abi, cpsat

import jobshop
import oracle_lib


class R:  # a MiLpResult stand-in
    def __init__(self, status, obj=0.0, err=0):
        self.problem_status, self.objective, self.error_code = status, obj, err


def _trail(n=4, obj_lb=10.0):
    return cpsat.IntegerTrail(np.zeros(n), np.ones(n) * 5, obj_lb=obj_lb)


def test_fold_branch_cases():
    # Lower branch infeasible: push var >= ceil(x), then the upper bound.
    t = _trail()
    lo = cpsat.BranchInfo(abi.DUAL_UNBOUNDED)
    up = cpsat.BranchInfo(abi.OPTIMAL, 12.3)
    assert cpsat.fold_branch(1, 2.5, lo, up, t)
    assert t.lb[1] == 3.0 and t.obj_lb == 13.0
    # Both infeasible: conflict.
    t = _trail()
    assert not cpsat.fold_branch(1, 2.5, cpsat.BranchInfo(abi.DUAL_UNBOUNDED),
                                 cpsat.BranchInfo(abi.DUAL_UNBOUNDED), t)
    assert t.conflict
    # No improvement on the lower branch: nothing, upper not consulted.
    t = _trail(obj_lb=20.0)
    assert not cpsat.fold_branch(1, 2.5, cpsat.BranchInfo(abi.OPTIMAL, 15.0), None, t)
    assert t.obj_lb == 20.0
    # Both improve: min of the two branch bounds (ceil(obj - 1e-4)).
    t = _trail()
    assert cpsat.fold_branch(0, 0.5, cpsat.BranchInfo(abi.OPTIMAL, 11.00005),
                             cpsat.BranchInfo(abi.DUAL_FEASIBLE, 14.2), t)
    assert t.obj_lb == 11.0
    # Upper branch infeasible: var <= floor(x), bound from the lower branch.
    t = _trail()
    assert cpsat.fold_branch(2, 3.7, cpsat.BranchInfo(abi.OPTIMAL, 16.5),
                             cpsat.BranchInfo(abi.DUAL_UNBOUNDED), t)
    assert t.ub[2] == 3.0 and t.obj_lb == 17.0
    # An unusable lower branch (ABNORMAL): no deduction.
    t = _trail()
    assert not cpsat.fold_branch(2, 3.7, cpsat.BranchInfo(abi.ABNORMAL), None, t)


def test_reduced_cost_strengthening():
    lp, ycols = jobshop.relaxation(jobshop.FT06)
    o = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=1))
    c = cpsat.LpConstraint(lp, ycols, o)
    t = cpsat.IntegerTrail(lp.col_lb, lp.col_ub, obj_ub=60.0)
    assert c.solve_lp(t)
    assert c.analyze_lp(t)
    assert t.obj_lb == math.ceil(c.lp_objective - cpsat.K_CP_EPSILON)
    # Every deduction is the reference's formula at the LP solution.
    t2 = cpsat.IntegerTrail(lp.col_lb, lp.col_ub, obj_ub=60.0)
    for col, kind, v in c.reduced_cost_deductions(t2, 60.0 - c.lp_objective):
        rc = c.reduced_costs[col]
        other = c.lp_solution[col] + (60.0 - c.lp_objective) / rc
        if kind == "le":
            assert rc > cpsat.K_LP_EPSILON and v == math.floor(other + cpsat.K_CP_EPSILON)
        else:
            assert rc < -cpsat.K_LP_EPSILON and v == math.ceil(other - cpsat.K_CP_EPSILON)


def _node(jobs, params):
    lp, ycols = jobshop.relaxation(jobs)
    o = oracle_lib.OracleLp(params)
    c = cpsat.LpConstraint(lp, ycols, o)
    t = cpsat.IntegerTrail(lp.col_lb, lp.col_ub)
    assert c.solve_lp(t) and c.analyze_lp(t)
    return lp, ycols, o, c, t


def test_batched_node_solves_the_branch_lps():
    """The batch call solves the LPs SolveLpForBranching solves: same
    bounds, same warm start (the node's state), same results bit for bit."""
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    lp, ycols, o, c, t = _node(jobshop.FT06, p)
    cols = cpsat.fractional_columns(c.lp_solution, ycols, limit=6)
    assert cols, "the ft06 root LP has fractional order variables"
    lbs, ubs = cpsat.branch_lps(t, c.lp_solution, cols)
    state = o.state()
    ws = [oracle_lib.OracleLp(p) for _ in range(3)]
    for w in ws:
        w.load(lp)
    batched = oracle_lib.batch_solve_bounds(ws, lbs, ubs, state)
    for i in range(len(lbs)):
        o.set_variable_bounds(lbs[i], ubs[i])
        info = c.solve_lp_for_branching()
        assert info.status == batched[i].problem_status
        if info.status in cpsat.KEEP_STATUSES:
            assert info.lp_objective == batched[i].objective
    o.set_variable_bounds(t.lb, t.ub)
    # The fold of the batch equals BranchOnVar run column by column from the
    # node's bounds (each column's first BranchOnVar call).
    ref = cpsat.IntegerTrail(t.lb, t.ub, t.obj_lb, t.obj_ub)
    summary = cpsat.fold_node(cpsat.IntegerTrail(t.lb, t.ub, t.obj_lb, t.obj_ub),
                              c.lp_solution, cols, batched)
    for col in cols:
        fresh = cpsat.IntegerTrail(t.lb, t.ub, ref.obj_lb, t.obj_ub)
        c.branch_on_var(col, fresh)
        ref.obj_lb = max(ref.obj_lb, fresh.obj_lb)
    assert summary["obj_lb"] == ref.obj_lb


@pytest.mark.gpu
def test_node_branch_lps_parity():
    """The engine's batched branch LPs (mi_lp_batch_solve_bounds, fibers and
    batched launches) against the oracle's, bit for bit, and the same fold."""
    import parity_util  # noqa: F401
    from mi_glop import engine
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    jobs = jobshop.random_instance(10, 5, 7)
    lp, ycols, o, c, t = _node(jobs, p)
    cols = cpsat.fractional_columns(c.lp_solution, ycols, limit=48)
    lbs, ubs = cpsat.branch_lps(t, c.lp_solution, cols)
    state = o.state()
    ws = [engine.LpHandle(p) for _ in range(16)]
    for w in ws:
        w.load(lp)
    got = engine.batch_solve_bounds(ws, lbs, ubs, state)
    os_ = [oracle_lib.OracleLp(p) for _ in range(4)]
    for w in os_:
        w.load(lp)
    ref = oracle_lib.batch_solve_bounds(os_, lbs, ubs, state)
    for a, b in zip(got, ref):
        assert (a.problem_status, a.error_code, a.iterations) == \
            (b.problem_status, b.error_code, b.iterations)
        assert a.objective == b.objective or (math.isnan(a.objective) and math.isnan(b.objective))
    s1 = cpsat.fold_node(cpsat.IntegerTrail(t.lb, t.ub, t.obj_lb), c.lp_solution, cols, got)
    s2 = cpsat.fold_node(cpsat.IntegerTrail(t.lb, t.ub, t.obj_lb), c.lp_solution, cols, ref)
    assert s1 == s2


def test_analyze_dual_feasible_reads_current_values():
    """AnalyzeLp on a DUAL_FEASIBLE result (the iteration cap hit by the dual
    simplex) deduces from the simplex's current reduced costs and values
    (linear_programming_constraint.cc:2380-2381), not from an earlier OPTIMAL
    solve, and pushes the objective bound first (:817-837)."""
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    lp, ycols, o, c, t = _node(jobshop.random_instance(6, 4, 3), p)
    stale_rc = c.reduced_costs.copy()
    cols = cpsat.fractional_columns(c.lp_solution, ycols, limit=1)
    assert cols
    lbs, ubs = cpsat.branch_lps(t, c.lp_solution, cols)
    trail = cpsat.IntegerTrail(lbs[0], ubs[0], obj_lb=t.obj_lb, obj_ub=t.obj_lb + 40.0)
    capped = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1)
    o.set_params(capped)
    assert c.solve_lp(trail)
    assert c.last.problem_status == abi.DUAL_FEASIBLE, abi.PROBLEM_STATUS[c.last.problem_status]
    rc, x = o.reduced_costs(), o.primal()
    assert not (np.array_equal(rc, stale_rc) and np.array_equal(x, c.lp_solution))
    want = []
    delta = (trail.obj_ub - c.last.objective) / lp.obj_scale
    for col in ycols:
        r = float(rc[col])
        if r == 0.0:
            continue
        other = float(x[col]) + delta / r
        if r > cpsat.K_LP_EPSILON and math.floor(other + cpsat.K_CP_EPSILON) < trail.ub[col]:
            want.append((int(col), "le", float(math.floor(other + cpsat.K_CP_EPSILON))))
        elif r < -cpsat.K_LP_EPSILON and math.ceil(other - cpsat.K_CP_EPSILON) > trail.lb[col]:
            want.append((int(col), "ge", float(math.ceil(other - cpsat.K_CP_EPSILON))))
    assert c.reduced_cost_deductions(trail, trail.obj_ub - c.last.objective) == want
    before_lb = trail.obj_lb
    ok = c.analyze_lp(trail)
    new_lb = math.ceil(c.last.objective - cpsat.K_CP_EPSILON)
    if ok:
        assert trail.obj_lb == max(before_lb, new_lb)
        for col, kind, v in want:
            assert (trail.ub[col] <= v) if kind == "le" else (trail.lb[col] >= v)


def test_propagate_iteration_caps_and_degeneracy():
    """Propagate's simplex caps (:1716-1723): root_lp_iterations at level 0,
    next_simplex_iter_ below; at linearization level 2 the limit follows
    UpdateSimplexIterationLimit with CalculateDegeneracy's count (:2351-2365)."""
    p = abi.default_params(use_dual_simplex=1)
    lp, ycols = jobshop.relaxation(jobshop.FT06)
    o = oracle_lib.OracleLp(p)
    c = cpsat.LpConstraint(lp, ycols, o, linearization_level=2)
    t = cpsat.IntegerTrail(lp.col_lb, lp.col_ub)
    assert c.propagate(t, level=0)
    assert o.params.max_number_of_iterations == cpsat.ROOT_LP_ITERATIONS
    assert c.last.problem_status == abi.OPTIMAL and c.lp_at_level_zero_is_final
    state = o.state()
    zero = np.concatenate([o.reduced_costs() == 0.0, o.duals() == 0.0])
    count = int(np.count_nonzero(zero & (np.asarray(state) != cpsat.BASIC)))
    assert c.calculate_degeneracy() == count
    assert c.is_degenerate == (count >= 0.3 * (lp.n + lp.m))
    cols = lp.n + lp.m
    if c.is_degenerate:
        expect = max(10, min(1000, 500 // max(1, 2 * ((10 * count) // cols))))
    else:
        expect = max(10, min(1000, cols // 40))
    assert c.next_simplex_iter == expect
    assert c.propagate(t, level=3)
    assert o.params.max_number_of_iterations == expect
