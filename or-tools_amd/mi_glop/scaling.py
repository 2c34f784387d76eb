"""LpScalingHelper (lp_data/lp_data_utils.h:51-83, .cc:76-182): the scaling
CP-SAT applies to its LP relaxation before handing it to the simplex
(sat/linear_programming_constraint.cc:417), and the conversions between the
original ("unscaled") problem and the scaled one.

Scale() runs the same passes as ScalingPreprocessor (SparseMatrixScaler,
LinearProgram::ScaleBounds, ScaleObjective) through the engine's host-only
entry point mi_lp_scale (engine.scale_lp). The factors kept are the
scaler's unscaling factors (row_scale_, col_scale_) and the reciprocals of the
bound and objective divisors, as the reference keeps them:

  bound_scaling_factor_     = 1 / lp->ScaleBounds()
  objective_scaling_factor_ = 1 / lp->ScaleObjective(cost_scaling)

Each conversion is the reference's formula, operation for operation (same
roundings), for one index or, vectorised, for a whole array.
"""
import numpy as np

from . import abi


class LpScalingHelper:
    def __init__(self):
        self.clear()

    def clear(self):
        """Clear (:85-89): every factor back to 1."""
        self.row_unscale = None  # SparseMatrixScaler::RowUnscalingFactor per row
        self.col_unscale = None  # ColUnscalingFactor per column
        self.bound_scaling_factor = 1.0
        self.objective_scaling_factor = 1.0

    def scale(self, lp, solver_params=None):
        """Scale (:78-83) with the GlopParameters subset of `solver_params`
        (abi.MiLpSolverParams; its scaling_method and cost_scaling). Returns the
        scaled copy of `lp` (the reference scales the LinearProgram in place)."""
        from . import engine
        sp = solver_params or abi.default_solver_params()
        # The helper scales whatever the preprocessing switch says.
        sp = abi.default_solver_params(use_scaling=1, scaling_method=sp.scaling_method,
                                       cost_scaling=sp.cost_scaling)
        scaled, f = engine.scale_lp(lp, sp)
        self.row_unscale = np.asarray(f["row_scale"], np.float64)
        self.col_unscale = np.asarray(f["col_scale"], np.float64)
        self.bound_scaling_factor = 1.0 / f["bound_factor"]
        self.objective_scaling_factor = 1.0 / f["cost_factor"]
        return scaled

    # -- factors ------------------------------------------------------------
    def _col(self, col):
        return 1.0 if self.col_unscale is None or col >= len(self.col_unscale) else \
            float(self.col_unscale[col])

    def _row(self, row):
        return 1.0 if self.row_unscale is None or row >= len(self.row_unscale) else \
            float(self.row_unscale[row])

    def _cols(self, n):
        return np.ones(n) if self.col_unscale is None else self.col_unscale[:n]

    def _rows(self, m):
        return np.ones(m) if self.row_unscale is None else self.row_unscale[:m]

    def variable_scaling_factor(self, col):
        """VariableScalingFactor (:91-95): original value x this = scaled."""
        return self._col(col) * self.bound_scaling_factor

    def bounds_scaling_factor(self):
        return self.bound_scaling_factor

    # -- unscaled -> scaled (:97-118) -------------------------------------------
    def scale_variable_value(self, col, value):
        return value * self._col(col) * self.bound_scaling_factor

    def scale_reduced_cost(self, col, value):
        return value / self._col(col) * self.objective_scaling_factor

    def scale_dual_value(self, row, value):
        return value * (self._row(row) * self.objective_scaling_factor)

    def scale_constraint_activity(self, row, value):
        return value / self._row(row) * self.bound_scaling_factor

    # -- scaled -> unscaled (:120-142) ------------------------------------------
    def unscale_variable_value(self, col, value):
        return value / (self._col(col) * self.bound_scaling_factor)

    def unscale_reduced_cost(self, col, value):
        return value * self._col(col) / self.objective_scaling_factor

    def unscale_dual_value(self, row, value):
        return value / (self._row(row) * self.objective_scaling_factor)

    def unscale_constraint_activity(self, row, value):
        return value * self._row(row) / self.bound_scaling_factor

    # -- whole arrays (the same formulas element-wise) ---------------------------
    def scale_variable_values(self, values):
        v = np.asarray(values, np.float64)
        return v * self._cols(len(v)) * self.bound_scaling_factor

    def unscale_variable_values(self, values):
        v = np.asarray(values, np.float64)
        return v / (self._cols(len(v)) * self.bound_scaling_factor)

    def unscale_reduced_costs(self, values):
        v = np.asarray(values, np.float64)
        return v * self._cols(len(v)) / self.objective_scaling_factor

    def unscale_dual_values(self, values):
        v = np.asarray(values, np.float64)
        return v / (self._rows(len(v)) * self.objective_scaling_factor)

    def unscale_constraint_activities(self, values):
        v = np.asarray(values, np.float64)
        return v * self._rows(len(v)) / self.bound_scaling_factor

    # -- solves (:144-182) ------------------------------------------------------
    def unscale_unit_row_left_solve(self, basis_col, values, non_zeros=None):
        """UnscaleUnitRowLeftSolve: left_inverse of [R B C] for the unit row
        of `basis_col`, in place (all entries, or the listed ones)."""
        g = self._col(basis_col)
        idx = range(len(values)) if non_zeros is None or len(non_zeros) == 0 else non_zeros
        for c in idx:
            values[c] /= self._row(c) * g
        return values

    def unscale_column_right_solve(self, basis, col, values, non_zeros=None):
        """UnscaleColumnRightSolve: B^-1 of column `col` of the scaled matrix,
        in place; `basis` maps rows to basic columns."""
        g = 1.0 / self._col(col)  # ColScalingFactor
        idx = range(len(values)) if non_zeros is None or len(non_zeros) == 0 else non_zeros
        for r in idx:
            values[r] /= self._col(int(basis[r])) * g
        return values
