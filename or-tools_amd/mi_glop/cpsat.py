"""CP-SAT's LP call-out over the engine.

Restates what sat/linear_programming_constraint.cc does around
RevisedSimplex for one LP constraint, on any solver handle with the engine's
surface (engine.LpHandle on the GPU; the tests drive the same code with the
CPU oracle):

* SolveLp (:709-760): solve with the trail's bounds, drop the warm start on
  an error, keep the matrix for the next solve, record the LP solution when
  OPTIMAL.
* AnalyzeLp (:762-860): a DUAL_UNBOUNDED LP is a conflict; an OPTIMAL or
  DUAL_FEASIBLE one pushes the objective lower bound ceil(obj - kCpEpsilon)
  and the reduced-cost strengthening deductions (:2367-2408).
* CalculateDegeneracy (:2351-2365) and UpdateSimplexIterationLimit
  (:1665-1695) for linearization level 2; Propagate (:1697-1806): the root
  cap root_lp_iterations = 2000 (sat_parameters.proto:899) at level 0, else
  next_simplex_iter_, then SolveLp and AnalyzeLp. Cut generation and the
  constraint manager's LP changes are CP-SAT search, out of scope: with no
  cut generators ChangeLp adds nothing, so one round ends the loop.
* BranchOnVar (:485-584) with SolveLpForBranching (:443-464): both branches of
  a fractional variable solved from the node's basis state, deductions from
  infeasible branches, the node's objective bound from the two branch bounds.
* The batched form of one search node (config 4): every branch LP of the
  node's fractional variables is solved at once (mi_lp_batch_solve_bounds,
  warm-started from the node's state, sharded over GPUs by the caller), then
  BranchOnVar's decisions are folded per variable in order. Upstream solves
  the branches one variable at a time and applies each variable's deductions
  before the next one; here every branch sees the node's bounds, so the
  branches are the LPs of the first BranchOnVar call per variable. An upper
  branch BranchOnVar would skip (lower branch not usable, or not improving)
  is solved anyway and counted as speculative.

Bounds are plain floats (the CP integer bounds). With scaling=False the LP
carries the CP variables unscaled (every scaler factor 1, the objective
scaling factor the LP's obj_scale). With scaling=True the LP is scaled once,
with its level-zero bounds, by LpScalingHelper (:417, scaling.py) under
CP-SAT's simplex parameters (MEAN_COST_SCALING, :234); the LP then sees bounds
times VariableScalingFactor (:699-707, :505-509), and the solution, reduced
costs and deductions are unscaled as at :685, :849 and :2367-2408.
"""
import ctypes
import math

import numpy as np

from . import abi
from .scaling import LpScalingHelper


def ctypes_copy(dst, src):
    ctypes.memmove(ctypes.addressof(dst), ctypes.addressof(src), ctypes.sizeof(src))

K_CP_EPSILON = 1e-4  # linear_programming_constraint.h:407
K_LP_EPSILON = 1e-6  # linear_programming_constraint.h:410
KEEP_STATUSES = (abi.OPTIMAL, abi.DUAL_FEASIBLE)
ROOT_LP_ITERATIONS = 2000  # sat_parameters.proto:899
BASIC = 0  # glop::VariableStatus::BASIC (lp_types.h), the state() encoding


class IntegerTrail:
    """The integer bounds a search node sees (IntegerTrail): per LP column a
    [lb, ub], plus the objective variable's [lb, ub] (objective_cp_)."""

    def __init__(self, col_lb, col_ub, obj_lb=-math.inf, obj_ub=math.inf):
        self.lb = np.array(col_lb, dtype=np.float64)
        self.ub = np.array(col_ub, dtype=np.float64)
        self.obj_lb = float(obj_lb)
        self.obj_ub = float(obj_ub)
        self.conflict = False

    def enqueue_ge(self, col, value):
        if value > self.ub[col]:
            self.conflict = True
            return False
        self.lb[col] = max(self.lb[col], value)
        return True

    def enqueue_le(self, col, value):
        if value < self.lb[col]:
            self.conflict = True
            return False
        self.ub[col] = min(self.ub[col], value)
        return True

    def enqueue_obj_ge(self, value):
        if value > self.obj_ub:
            self.conflict = True
            return False
        self.obj_lb = max(self.obj_lb, value)
        return True


class BranchInfo:
    """LPSolveInfo of one branch (linear_programming_constraint.h)."""

    def __init__(self, status, lp_objective=math.nan):
        self.status = status
        self.lp_objective = lp_objective
        self.new_obj_bound = -math.inf
        if status in KEEP_STATUSES:
            self.new_obj_bound = float(math.ceil(lp_objective - K_CP_EPSILON))


class LpConstraint:
    """One LinearProgrammingConstraint: an LP over the columns `int_cols`
    (integer variables) of `lp`, solved by `handle` (engine.LpHandle or a
    handle with the same surface)."""

    def __init__(self, lp, int_cols, handle, linearization_level=1, scaling=False):
        self.lp = lp
        self.int_cols = np.asarray(int_cols, dtype=np.int64)
        self.h = handle
        self.scaler = LpScalingHelper()
        self.lp_data = lp  # what the simplex holds (lp_data_)
        if scaling:
            self.lp_data = self.scaler.scale(
                lp, abi.default_solver_params(cost_scaling=abi.MEAN_COST_SCALING))
        # VariableScalingFactor of every column (1 without scaling).
        self.factor = np.array([self.scaler.variable_scaling_factor(c) for c in range(lp.n)])
        self.h.load(self.lp_data)
        self.linearization_level = linearization_level
        self.next_simplex_iter = 500  # linear_programming_constraint.h:548
        self.is_degenerate = False
        self.lp_at_level_zero_is_final = False
        self.lp_solution = None
        self.lp_objective = math.nan
        self.reduced_costs = None
        self.num_solves = 0
        self.total_iterations = 0

    # -- SolveLp (:709-760) -------------------------------------------------
    def scale_bounds(self, lbs, ubs):
        """CP bounds -> the LP's (times VariableScalingFactor, :704-705); rows
        of a 2-D array are independent bound sets (branch_lps)."""
        return np.asarray(lbs) * self.factor, np.asarray(ubs) * self.factor

    def update_bounds(self, trail):
        """UpdateBoundsOfLpVariables (:699-707)."""
        self.h.set_variable_bounds(*self.scale_bounds(trail.lb, trail.ub))

    def solve_lp(self, trail):
        self.update_bounds(trail)
        r = self.h.solve()
        self.total_iterations += int(r.iterations)
        self.last = r
        if r.error_code != 0:
            self.h.clear_basis_state()
            return False
        self.h.notify_matrix_unchanged()
        self.num_solves += 1
        if r.problem_status == abi.OPTIMAL:
            # GetVariableValueAtCpScale (:683-686)
            self.lp_solution = self.scaler.unscale_variable_values(self.h.primal())
        return True

    # -- Propagate (:1697-1806) ----------------------------------------------
    def set_iteration_cap(self, level):
        """The simplex iteration cap Propagate sets (:1716-1723)."""
        cap = ROOT_LP_ITERATIONS if level == 0 else self.next_simplex_iter
        p = type(self.h.params)()
        ctypes_copy(p, self.h.params)
        p.max_number_of_iterations = int(cap)
        self.h.set_params(p)
        return cap

    def propagate(self, trail, level=0):
        """One Propagate call at decision level `level`. Returns False on a
        conflict. The cut loop (:1731-1806) adds nothing here (no cut
        generators), which ends it after the first round; at level 0 that
        marks the level-zero LP final (:1797-1800)."""
        self.set_iteration_cap(level)
        if not self.solve_lp(trail):
            return True
        if not self.analyze_lp(trail):
            return False
        if self.last.problem_status == abi.OPTIMAL and level == 0:
            self.lp_at_level_zero_is_final = True
        return True

    def calculate_degeneracy(self):
        """CalculateDegeneracy (:2351-2365): non-basic columns (slacks
        included: RevisedSimplex's num_cols_) with a zero reduced cost; a slack's
        reduced cost is minus its row's dual value."""
        state = np.asarray(self.h.state())
        n = self.lp.n
        zero = np.concatenate([np.asarray(self.h.reduced_costs())[:n] == 0.0,
                               np.asarray(self.h.duals()) == 0.0])
        count = int(np.count_nonzero(zero & (state != BASIC)))
        self.is_degenerate = count >= 0.3 * len(state)
        return count

    # -- AnalyzeLp (:762-860) ------------------------------------------------
    def analyze_lp(self, trail):
        """Returns False on a conflict (infeasible LP, or a bound crossing).
        The deductions read the simplex's current reduced costs and values
        (GetReducedCost / GetVariableValue, :2380-2381) for OPTIMAL and
        DUAL_FEASIBLE alike; the objective bound is pushed before them
        (:817-837)."""
        r = self.last
        if r.problem_status == abi.DUAL_UNBOUNDED:
            trail.conflict = True
            return False
        self.update_iteration_limit(r.problem_status)
        if r.problem_status in KEEP_STATUSES:
            obj = float(r.objective)
            rc = np.asarray(self.h.reduced_costs())
            x = np.asarray(self.h.primal())
            deductions = self.reduced_cost_deductions(trail, trail.obj_ub - obj, rc, x)
            new_lb = float(math.ceil(obj - K_CP_EPSILON))
            if new_lb > trail.obj_lb and not trail.enqueue_obj_ge(new_lb):
                return False
            for col, kind, value in deductions:
                ok = trail.enqueue_le(col, value) if kind == "le" else trail.enqueue_ge(col, value)
                if not ok:
                    return False
        if r.problem_status == abi.OPTIMAL:
            self.lp_objective = float(r.objective)
            self.reduced_costs = self.scaler.unscale_reduced_costs(self.h.reduced_costs())
        return True

    def reduced_cost_deductions(self, trail, cp_objective_delta, rc=None, x=None):
        """ReducedCostStrengtheningDeductions (:2367-2408): a column moved off
        its bound by more than objective slack / |rc| would cross the
        incumbent. rc and x default to the handle's current values."""
        out = []
        if not math.isfinite(cp_objective_delta):
            return out
        # TRICKY (:2370-2374): only the objective value carries the LP's
        # objective scaling factor; rc and x are the simplex's own.
        lp_delta = cp_objective_delta / self.lp_data.obj_scale
        rc = np.asarray(self.h.reduced_costs()) if rc is None else rc
        x = np.asarray(self.h.primal()) if x is None else x
        for col in self.int_cols:
            c = float(rc[col])
            if c == 0.0:
                continue
            other = self.scaler.unscale_variable_value(int(col), float(x[col]) + lp_delta / c)
            if c > K_LP_EPSILON:
                new_ub = math.floor(other + K_CP_EPSILON)
                if new_ub < trail.ub[col]:
                    out.append((int(col), "le", float(new_ub)))
            elif c < -K_LP_EPSILON:
                new_lb = math.ceil(other - K_CP_EPSILON)
                if new_lb > trail.lb[col]:
                    out.append((int(col), "ge", float(new_lb)))
        return out

    def update_iteration_limit(self, status, min_iter=10, max_iter=1000):
        """UpdateSimplexIterationLimit (:1665-1695); level < 2 keeps it."""
        if self.linearization_level < 2:
            return
        num_degenerate_columns = self.calculate_degeneracy()
        num_cols = self.lp.n + self.lp.m  # GetProblemNumCols (slacks included)
        if num_cols <= 0:
            return
        decrease = (10 * num_degenerate_columns) // num_cols
        degenerate = self.is_degenerate
        if status == abi.DUAL_FEASIBLE:
            if degenerate:
                self.next_simplex_iter //= max(1, decrease)
            else:
                self.next_simplex_iter *= 2
        elif status == abi.OPTIMAL:
            if degenerate:
                self.next_simplex_iter //= max(1, 2 * decrease)
            else:
                self.next_simplex_iter = num_cols // 40
        self.next_simplex_iter = max(min_iter, min(max_iter, self.next_simplex_iter))

    # -- BranchOnVar (:485-584) ----------------------------------------------
    def solve_lp_for_branching(self):
        """SolveLpForBranching (:443-464): solve, then restore the state the
        node had (the branches are explored from the node's basis)."""
        state = self.h.state()
        r = self.h.solve()
        self.total_iterations += int(r.iterations)
        self.h.load_basis_state(state)
        if r.error_code != 0:
            return BranchInfo(abi.ABNORMAL)
        return BranchInfo(int(r.problem_status), float(r.objective))

    def branch_on_var(self, col, trail):
        """The sequential BranchOnVar of one fractional column; returns
        whether a deduction was made."""
        value = float(self.lp_solution[col])
        lb, ub = float(trail.lb[col]), float(trail.ub[col])
        if value < lb or value > ub:
            return False
        self.update_bounds(trail)
        lbs = trail.lb.copy()
        ubs = trail.ub.copy()
        ubs[col] = math.floor(value)
        self.h.set_variable_bounds(*self.scale_bounds(lbs, ubs))
        lower = self.solve_lp_for_branching()
        ubs[col] = ub
        lbs[col] = math.ceil(value)
        upper = None
        if _usable(lower) and not (lower.status != abi.DUAL_UNBOUNDED and
                                   lower.new_obj_bound <= trail.obj_lb):
            self.h.set_variable_bounds(*self.scale_bounds(lbs, ubs))
            upper = self.solve_lp_for_branching()
        self.update_bounds(trail)
        return fold_branch(col, value, lower, upper, trail)


def _usable(info):
    return info.status in (abi.OPTIMAL, abi.DUAL_FEASIBLE, abi.DUAL_UNBOUNDED)


def fold_branch(col, value, lower, upper, trail):
    """BranchOnVar's decisions (:510-583) from the two branch results (upper
    is None when the sequential code would not have solved it)."""
    deductions = False
    if not _usable(lower):
        return False
    if lower.status == abi.DUAL_UNBOUNDED:
        if not trail.enqueue_ge(col, math.ceil(value)):
            return False
        deductions = True
    elif lower.new_obj_bound <= trail.obj_lb:
        return False
    if upper is None or not _usable(upper):
        return deductions
    if upper.status == abi.DUAL_UNBOUNDED:
        if lower.status != abi.DUAL_UNBOUNDED:
            if not trail.enqueue_le(col, math.floor(value)):
                return deductions
            deductions = True
    elif upper.new_obj_bound <= trail.obj_lb:
        return deductions
    if lower.status == abi.DUAL_UNBOUNDED and upper.status == abi.DUAL_UNBOUNDED:
        trail.conflict = True
        return False
    if lower.status == abi.DUAL_UNBOUNDED:
        approx = upper.new_obj_bound
    elif upper.status == abi.DUAL_UNBOUNDED:
        approx = lower.new_obj_bound
    else:
        approx = min(lower.new_obj_bound, upper.new_obj_bound)
    if approx <= trail.obj_lb:
        return deductions
    if not trail.enqueue_obj_ge(approx):
        return deductions
    return True


# --- the batched search node (config 4) ---------------------------------------

def fractional_columns(x, int_cols, limit=None):
    """The LP solution's fractional integer columns (|x - round(x)| >
    kCpEpsilon, the test of AnalyzeLp :848-852), most fractional first, ties
    by column."""
    x = np.asarray(x)
    frac = [(abs(x[c] - round(x[c])), int(c)) for c in int_cols
            if abs(x[c] - round(x[c])) > K_CP_EPSILON]
    frac.sort(key=lambda t: (-min(t[0], 1.0 - t[0]), t[1]))
    cols = [c for _, c in frac]
    return cols if limit is None else cols[:limit]


def branch_lps(trail, x, cols):
    """The two branch LPs (var <= floor(x), var >= ceil(x)) of every column,
    as (lbs, ubs) arrays of 2 * len(cols) rows: down branch, then up, per
    column in order."""
    k = len(cols)
    lbs = np.repeat(trail.lb[None, :], 2 * k, axis=0)
    ubs = np.repeat(trail.ub[None, :], 2 * k, axis=0)
    for i, c in enumerate(cols):
        ubs[2 * i, c] = math.floor(x[c])
        lbs[2 * i + 1, c] = math.ceil(x[c])
    return lbs, ubs


def fold_node(trail, x, cols, results):
    """Folds batched branch results (MiLpResult per branch LP, in branch_lps
    order) with BranchOnVar's decisions, column by column. Returns a summary:
    deductions made, the node's objective lower bound, speculative LPs (upper
    branches the sequential code would have skipped), conflict."""
    deduced = 0
    speculative = 0
    for i, c in enumerate(cols):
        lo, up = results[2 * i], results[2 * i + 1]
        lower = BranchInfo(int(lo.problem_status), float(lo.objective)) \
            if lo.error_code == 0 else BranchInfo(abi.ABNORMAL)
        upper = BranchInfo(int(up.problem_status), float(up.objective)) \
            if up.error_code == 0 else BranchInfo(abi.ABNORMAL)
        skip_upper = (not _usable(lower)) or (lower.status != abi.DUAL_UNBOUNDED and
                                              lower.new_obj_bound <= trail.obj_lb)
        if skip_upper:
            speculative += 1
        if fold_branch(c, float(x[c]), lower, None if skip_upper else upper, trail):
            deduced += 1
        if trail.conflict:
            break
    return {"deductions": deduced, "obj_lb": trail.obj_lb, "speculative": speculative,
            "conflict": trail.conflict}
