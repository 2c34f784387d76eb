"""TEST INFRASTRUCTURE ONLY (the checker, never the product): a numpy
restatement of Glop's scaling preprocessor and of the value part of
LPSolver's solution recovery, against which the engine's LPSolver layer
(or-tools_amd/csrc/engine/lp_solver.cc, C ABI mi_lp_scale /
mi_lp_solver_solve) is compared bit for bit.

Followed, operation by operation:
  * SparseMatrixScaler::Scale and its passes, lp_data/matrix_scaler.cc
    (ComputeMinAndMaxMagnitudes sparse.cc:375-393; 4 geometric iterations
    with the variance stop at 10; EquilibrateRows / EquilibrateColumns);
  * lp_data_utils.cc Scale(): c /= C, bounds *= C, row bounds /= R;
  * LinearProgram::ScaleObjective / ScaleBounds, lp_data.cc:1144-1258;
  * ScalingPreprocessor::RecoverSolution, glop/preprocessor.cc:3878-3912;
  * LPSolver::LoadAndVerifySolution value part, glop/lp_solver.cc:334-367,
    540-579, 866-896 (AccurateSum of base/accurate_sum.h:23-42).
Sums that Glop accumulates left to right are accumulated left to right here
(np.cumsum or plain loops, never np.sum's pairwise tree).
Parity pinned by the reference only at the objective level: the known-answer
LPs of tests/kat_lps.py solved through this layer must reach the objectives
the reference's tests state.
"""
import math

import numpy as np

INF = math.inf


def _seq_sum(a):
    return float(np.cumsum(a)[-1]) if len(a) else 0.0


class Scaler:
    def __init__(self, m, n, starts, rows, vals):
        self.m, self.n = m, n
        self.starts = np.asarray(starts, np.int64)
        self.rows = np.asarray(rows, np.int64)
        self.vals = np.array(vals, np.float64)
        self.row_scale = np.ones(m)
        self.col_scale = np.ones(n)

    def _min_max(self):
        a = np.abs(self.vals)
        a = a[a != 0.0]
        if len(a) == 0:
            return 0.0, 0.0
        return float(a.min()), float(a.max())

    def _variance(self):
        a = np.abs(self.vals)
        a = a[a != 0.0]
        if len(a) == 0:
            return 0.0
        sq = _seq_sum(a * a)
        ab = _seq_sum(a)
        n = float(len(a))
        return (sq - ab * ab / n) / n

    def _scale_rows(self, f):
        scaled = int(np.count_nonzero(f != 1.0))
        self.row_scale = np.where(f != 1.0, self.row_scale * f, self.row_scale)
        self.vals = self.vals / f[self.rows]
        return scaled

    def _col_ranges(self):
        for c in range(self.n):
            yield c, slice(self.starts[c], self.starts[c + 1])

    def _rows_geometric(self):
        a = np.abs(self.vals)
        nz = a != 0.0
        mx = np.zeros(self.m)
        mn = np.full(self.m, INF)
        np.maximum.at(mx, self.rows[nz], a[nz])
        np.minimum.at(mn, self.rows[nz], a[nz])
        f = np.where(mx == 0.0, 1.0, np.sqrt(np.where(mx == 0.0, 1.0, mx * mn)))
        return self._scale_rows(f)

    def _cols_geometric(self):
        scaled = 0
        for c, sl in self._col_ranges():
            a = np.abs(self.vals[sl])
            a = a[a != 0.0]
            if len(a):
                f = math.sqrt(float(a.max()) * float(a.min()))
                self.col_scale[c] *= f
                self.vals[sl] = self.vals[sl] / f
                scaled += 1
        return scaled

    def _equilibrate_rows(self):
        a = np.abs(self.vals)
        nz = a != 0.0
        mx = np.zeros(self.m)
        np.maximum.at(mx, self.rows[nz], a[nz])
        mx[mx == 0.0] = 1.0
        return self._scale_rows(mx)

    def _equilibrate_cols(self):
        for c, sl in self._col_ranges():
            if sl.stop > sl.start:
                mx = float(np.abs(self.vals[sl]).max())
                if mx != 0.0:
                    self.col_scale[c] *= mx
                    self.vals[sl] = self.vals[sl] / mx

    def scale(self):
        mn, mx = self._min_max()
        if mn == 0.0:
            return
        if mx / mn < 1e20:
            for _ in range(4):
                r = self._rows_geometric()
                c = self._cols_geometric()
                if self._variance() < 10.0 or (r == 0 and c == 0):
                    break
        self._equilibrate_rows()
        self._equilibrate_cols()


def _update_min_max(v, mn, mx):
    a = np.abs(np.asarray(v, np.float64))
    a = a[(a != 0) & (a != INF)]
    if len(a):
        mn = min(mn, float(a.min()))
        mx = max(mx, float(a.max()))
    return mn, mx


def _divisor(mn, mx):
    if 1.0 < mn < INF:
        return mn
    if 0.0 < mx < 1.0:
        return mx
    return 1.0


def scale_lp(lp, cost_scaling=1, use_scaling=True):
    """ScalingPreprocessor::Run on a copy: returns (arrays dict, factors dict)."""
    s = Scaler(lp.m, lp.n, lp.col_starts, lp.row_idx, lp.vals)
    obj = np.array(lp.obj, np.float64)
    clb, cub = np.array(lp.col_lb, np.float64), np.array(lp.col_ub, np.float64)
    rlb, rub = np.array(lp.row_lb, np.float64), np.array(lp.row_ub, np.float64)
    offset, oscale = float(lp.obj_offset), float(lp.obj_scale)
    cf = bf = 1.0
    if use_scaling:
        s.scale()
        obj = obj / s.col_scale
        cub = cub * s.col_scale
        clb = clb * s.col_scale
        rub = rub / s.row_scale
        rlb = rlb / s.row_scale
        mn, mx = _update_min_max(obj, INF, 0.0)
        if cost_scaling == 1:
            cf = _divisor(mn, mx)
        elif cost_scaling == 2:
            nz = np.abs(obj[obj != 0.0])
            cf = _seq_sum(nz) / float(len(nz)) if len(nz) else 1.0
        elif cost_scaling == 3:
            nz = np.sort(np.abs(obj[obj != 0.0]))
            cf = float(nz[len(nz) // 2]) if len(nz) else 1.0
        if cf != 1.0:
            obj = np.where(obj == 0.0, obj, obj / cf)
            oscale = oscale * cf
            offset = offset / cf
        mn, mx = INF, 0.0
        for v in (clb, cub, rlb, rub):
            mn, mx = _update_min_max(v, mn, mx)
        bf = _divisor(mn, mx)
        if bf != 1.0:
            oscale = oscale * bf
            offset = offset / bf
            clb, cub, rlb, rub = clb / bf, cub / bf, rlb / bf, rub / bf
    arrays = dict(vals=s.vals, obj=obj, col_lb=clb, col_ub=cub, row_lb=rlb, row_ub=rub,
                  obj_offset=offset, obj_scale=oscale)
    return arrays, dict(row_scale=s.row_scale, col_scale=s.col_scale, cost_factor=cf,
                        bound_factor=bf)


# glop::VariableStatus (lp_types.h:188-199)
BASIC, FIXED_VALUE, AT_LOWER, AT_UPPER, FREE = range(5)


def recover_and_verify(lp, factors, x, y, vstat, status_optimal, strong=True,
                       use_scaling=True):
    """RecoverSolution + LoadAndVerifySolution value part on the original LP.
    Returns dict(x, y, rc, act, objective)."""
    x = np.array(x, np.float64)
    y = np.array(y, np.float64)
    clb, cub = np.asarray(lp.col_lb, np.float64), np.asarray(lp.col_ub, np.float64)
    if use_scaling:
        x = x / factors["col_scale"] * factors["bound_factor"]
        y = y / factors["row_scale"] * factors["cost_factor"]
        vs = np.asarray(vstat)
        x = np.where((vs == AT_UPPER) | (vs == FIXED_VALUE), cub, x)
        x = np.where(vs == AT_LOWER, clb, x)
    if strong and status_optimal:
        x = np.maximum(np.minimum(x, cub), clb)
        sign = -1.0 if lp.maximize else 1.0
        d = sign * y
        d = np.where((np.asarray(lp.row_lb) == -INF) & (d > 0.0), 0.0, d)
        d = np.where((np.asarray(lp.row_ub) == INF) & (d < 0.0), 0.0, d)
        y = sign * d
    s = e = 0.0
    for c in range(lp.n):  # AccurateSum
        e += float(lp.obj[c]) * float(x[c])
        t = s + e
        e += s - t
        s = t
    objective = float(lp.obj_scale) * (s + float(lp.obj_offset))
    rc = np.zeros(lp.n)
    act = np.zeros(lp.m)
    for c in range(lp.n):
        lo, hi = int(lp.col_starts[c]), int(lp.col_starts[c + 1])
        dot = 0.0
        for k in range(lo, hi):
            dot += float(y[lp.row_idx[k]]) * float(lp.vals[k])
        rc[c] = float(lp.obj[c]) - dot
        if x[c] != 0.0:
            for k in range(lo, hi):
                act[lp.row_idx[k]] += float(x[c]) * float(lp.vals[k])
    return dict(x=x, y=y, rc=rc, act=act, objective=objective)
