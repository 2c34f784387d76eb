#!/usr/bin/env python3
"""Development aid: writes the U^T factor saved by scripts/analyze_u.py (npz)
and a seeded dense right-hand side in tri_bench's binary format:
int32 n, int64 nnz, int64 starts[n+1], int32 rows[nnz], double vals[nnz],
double diag[n], double rhs[n]. Columns of U^T (= rows of U) hold rows j > c in
increasing order, as TriangularMatrix::PopulateFromTranspose leaves them."""
import sys

import numpy as np

src, dst = sys.argv[1], sys.argv[2]
z = np.load(src)
starts, rows, vals, diag = z["starts"], z["rows"], z["vals"], z["diag"]
n = len(starts) - 1
cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(starts))
# U(i, j): column j, row i < j.  U^T column i holds (j, U(i, j)), j ascending.
order = np.lexsort((cols, rows))
t_rows = cols[order].astype(np.int32)
t_vals = vals[order]
t_starts = np.zeros(n + 1, np.int64)
np.cumsum(np.bincount(rows, minlength=n), out=t_starts[1:])
rhs = np.random.default_rng(7).uniform(-1, 1, size=n)
with open(dst, "wb") as f:
    np.array([n], np.int32).tofile(f)
    np.array([len(t_rows)], np.int64).tofile(f)
    t_starts.tofile(f)
    t_rows.tofile(f)
    t_vals.tofile(f)
    diag.astype(np.float64).tofile(f)
    rhs.tofile(f)
print(f"n {n} nnz {len(t_rows)} -> {dst}")
