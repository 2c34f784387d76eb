#!/usr/bin/env python3
"""Development aid: the structure of config 5's U factor at the bench window.

Runs the oracle (CPU) on the config-5 LP to an iteration cap, exports the
current LU's U (oracle_lp_debug_upper) and prints the dependency levels of
the dense U solve (TransposeLowerSolve of U^T, sparse.cc:899-955: output i
reads x[j] for every U(i, j) != 0, j > i): critical path, widths, entries
per level. Saves the factor to --save (npz) for kernel-design experiments."""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "or-tools_amd"), os.path.join(REPO, "tests")]

from mi_glop import abi  # noqa: E402
import lp_gen  # noqa: E402
import oracle_lib  # noqa: E402


def export_upper(o):
    L = oracle_lib.lib()
    vp = ctypes.c_void_p
    L.oracle_lp_debug_upper.argtypes = [vp] * 6
    sizes = np.zeros(2, np.int64)
    L.oracle_lp_debug_upper(o.h, sizes.ctypes.data_as(vp), None, None, None, None)
    n, nnz = int(sizes[0]), int(sizes[1])
    starts = np.zeros(n + 1, np.int64)
    rows = np.zeros(nnz, np.int32)
    vals = np.zeros(nnz)
    diag = np.zeros(n)
    L.oracle_lp_debug_upper(o.h, sizes.ctypes.data_as(vp), starts.ctypes.data_as(vp),
                            rows.ctypes.data_as(vp), vals.ctypes.data_as(vp),
                            diag.ctypes.data_as(vp))
    return starts, rows, vals, diag


def levels_of(starts, rows):
    """level[i] = 1 + max level[j] over U(i, j) != 0 (j > i); 0 without entries."""
    n = len(starts) - 1
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(starts))
    # Process outputs from the last to the first (every j > i is final).
    order = np.argsort(rows, kind="stable")
    r_sorted = rows[order]
    c_sorted = cols[order]
    bounds = np.searchsorted(r_sorted, np.arange(n + 1))
    level = np.zeros(n, np.int64)
    for i in range(n - 1, -1, -1):
        a, b = bounds[i], bounds[i + 1]
        if b > a:
            level[i] = 1 + level[c_sorted[a:b]].max()
    per_row = np.diff(bounds)
    return level, per_row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=100000)
    ap.add_argument("--n", type=int, default=1000000)
    ap.add_argument("--cap", type=int, default=20005)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--save", default="")
    a = ap.parse_args()
    lp = lp_gen.sparse_c5_lp(a.m, a.n, 10, a.seed)
    o = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=1, max_number_of_iterations=a.cap))
    o.load(lp)
    t = time.time()
    r = o.solve()
    print(f"oracle: {r.iterations} iterations in {time.time() - t:.1f}s", flush=True)
    starts, rows, vals, diag = export_upper(o)
    n = len(starts) - 1
    level, per_row = levels_of(starts, rows)
    L = int(level.max()) + 1
    width = np.bincount(level, minlength=L)
    ent = np.bincount(level, weights=per_row, minlength=L)
    print(f"U: {n} columns, {len(rows)} off-diagonal entries, {L} levels, "
          f"unit diagonal {bool(np.all(diag == 1.0))}")
    print(f"rows with entries: {(per_row > 0).sum()}, max entries/row {per_row.max()}, "
          f">4: {(per_row > 4).sum()}")
    for lv in range(L):
        print(f"  level {lv:4d}: width {width[lv]:7d} entries {int(ent[lv]):8d}")
    if a.save:
        np.savez(a.save, starts=starts, rows=rows, vals=vals, diag=diag, level=level)


if __name__ == "__main__":
    main()
