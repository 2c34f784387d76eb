"""In-memory LP in the shape Glop's RevisedSimplex::Solve consumes.

Mirrors the subset of glop::LinearProgram (ortools/lp_data/lp_data.h:56) the
revised simplex reads: A in CSC with rows sorted per column and no explicit
zeros (LinearProgram::IsCleanedUp, lp_solver.cc:185-191), variable and
constraint bounds, objective, offset, scaling factor and sense.
"""
from dataclasses import dataclass, field

import numpy as np

INF = np.inf


@dataclass
class LinearProgram:
    m: int
    n: int
    col_starts: np.ndarray  # int64[n+1]
    row_idx: np.ndarray  # int32[nnz]
    vals: np.ndarray  # float64[nnz]
    col_lb: np.ndarray
    col_ub: np.ndarray
    row_lb: np.ndarray
    row_ub: np.ndarray
    obj: np.ndarray
    obj_offset: float = 0.0
    obj_scale: float = 1.0
    maximize: bool = False
    name: str = field(default="lp")

    @property
    def nnz(self):
        return int(self.col_starts[-1])

    def validate(self):
        """LinearProgram::IsValid / IsCleanedUp checks (lp_solver.cc:185-202)."""
        cs = self.col_starts
        if cs.shape != (self.n + 1,) or cs[0] != 0 or np.any(np.diff(cs) < 0):
            return False
        for c in range(self.n):
            r = self.row_idx[cs[c]:cs[c + 1]]
            if np.any(np.diff(r) <= 0):
                return False
        if np.any(self.row_idx < 0) or np.any(self.row_idx >= self.m):
            return False
        if np.any(self.vals == 0) or not np.all(np.isfinite(self.vals)):
            return False
        for lo, hi in ((self.col_lb, self.col_ub), (self.row_lb, self.row_ub)):
            if np.any(lo > hi) or np.any(lo == INF) or np.any(hi == -INF):
                return False
        return bool(np.all(np.isfinite(self.obj)))

    @staticmethod
    def from_dense(A, col_lb, col_ub, row_lb, row_ub, obj, offset=0.0,
                   maximize=False, name="lp"):
        A = np.asarray(A, dtype=np.float64)
        m, n = A.shape
        starts = [0]
        rows, vals = [], []
        for c in range(n):
            nz = np.nonzero(A[:, c])[0]
            rows.extend(nz.tolist())
            vals.extend(A[nz, c].tolist())
            starts.append(len(rows))
        return LinearProgram(
            m, n, np.asarray(starts, np.int64), np.asarray(rows, np.int32),
            np.asarray(vals, np.float64), np.asarray(col_lb, np.float64),
            np.asarray(col_ub, np.float64), np.asarray(row_lb, np.float64),
            np.asarray(row_ub, np.float64), np.asarray(obj, np.float64),
            float(offset), 1.0, bool(maximize), name)

    @staticmethod
    def from_triplets(m, n, triplets, col_lb, col_ub, row_lb, row_ub, obj,
                      offset=0.0, maximize=False, name="lp"):
        A = np.zeros((m, n))
        for r, c, v in triplets:
            A[r, c] = v
        return LinearProgram.from_dense(A, col_lb, col_ub, row_lb, row_ub, obj,
                                        offset, maximize, name)
