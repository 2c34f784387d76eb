"""Optimality check of a basic solution that does not go through the Glop
restatement (test infrastructure): the KKT conditions of

    min / max  c.x   s.t.  row_lb <= A x <= row_ub,  col_lb <= x <= col_ub

computed in numpy from the LP and a solver's primal values, duals, reduced
costs and statuses, with Glop's sign conventions (rc = c - A^T y; for a
minimization a column at its lower bound has rc >= 0, at its upper bound
rc <= 0, a basic one rc = 0; a constraint at its lower bound has y >= 0, at
its upper bound y <= 0, a basic one y = 0; VariableStatus values
lp_types.h:192-219). Used by tests/test_independent_gpu.py and
scripts/whole_solve.py next to the bit-for-bit oracle checks, so that a
misreading shared by the engine and the oracle (a fork of one another)
would still show."""
import numpy as np

BASIC, FIXED, AT_LOWER, AT_UPPER, FREE = 0, 1, 2, 3, 4


def kkt(lp, x, y, rc, vstat, cstat, maximize=False):
    """Max violations: primal bounds, rows (relative to max |x|), the
    reduced-cost identity, and the dual sign conditions of columns and rows;
    plus the primal objective c.x (without the offset)."""
    n, m = lp.n, lp.m
    cs = np.asarray(lp.col_starts)
    cols = np.repeat(np.arange(n), np.diff(cs))
    rows = np.asarray(lp.row_idx)
    vals = np.asarray(lp.vals)
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    rc = np.asarray(rc, dtype=np.float64)
    vstat = np.asarray(vstat)
    cstat = np.asarray(cstat)
    ax = np.zeros(m)
    np.add.at(ax, rows, vals * x[cols])
    aty = np.zeros(n)
    np.add.at(aty, cols, vals * y[rows])
    obj = np.asarray(lp.obj)
    scale = max(1.0, float(np.abs(x).max(initial=0.0)))
    out = {
        "primal_bound_violation": float(max(np.max(np.asarray(lp.col_lb) - x, initial=0.0),
                                            np.max(x - np.asarray(lp.col_ub), initial=0.0))),
        "row_violation": float(max(np.max(np.asarray(lp.row_lb) - ax, initial=0.0),
                                   np.max(ax - np.asarray(lp.row_ub), initial=0.0))) / scale,
        "rc_identity": float(np.max(np.abs(rc - (obj - aty)), initial=0.0)),
    }
    sgn = -1.0 if maximize else 1.0
    r = sgn * rc
    bad_col = np.zeros(n)
    bad_col[vstat == AT_LOWER] = np.maximum(0.0, -r[vstat == AT_LOWER])
    bad_col[vstat == AT_UPPER] = np.maximum(0.0, r[vstat == AT_UPPER])
    bad_col[vstat == BASIC] = np.abs(r[vstat == BASIC])
    bad_col[vstat == FREE] = np.abs(r[vstat == FREE])
    yy = sgn * y
    bad_row = np.zeros(m)
    bad_row[cstat == AT_LOWER] = np.maximum(0.0, -yy[cstat == AT_LOWER])
    bad_row[cstat == AT_UPPER] = np.maximum(0.0, yy[cstat == AT_UPPER])
    bad_row[cstat == BASIC] = np.abs(yy[cstat == BASIC])
    out["dual_sign_violation_cols"] = float(bad_col.max(initial=0.0))
    out["dual_sign_violation_rows"] = float(bad_row.max(initial=0.0))
    out["primal_objective"] = float(obj @ x)
    return out


def assert_optimal(lp, x, y, rc, vstat, cstat, tol=1e-6):
    k = kkt(lp, x, y, rc, vstat, cstat, bool(lp.maximize))
    for key in ("primal_bound_violation", "row_violation", "rc_identity",
                "dual_sign_violation_cols", "dual_sign_violation_rows"):
        assert k[key] <= tol, (key, k)
    return k
