"""Seeded synthetic LP generators (BASELINE.md section 2 / SURVEY.md 8(d)).

All generators are deterministic functions of (shape, seed).
"""
import numpy as np

from mi_glop.lp import LinearProgram

INF = np.inf


def random_sparse_lp(m, n, density, seed, eq_frac=0.2, free_frac=0.05,
                     boxed_frac=0.5, maximize=False):
    """Feasible LP with mixed row/column bound types (exercises every
    VariableType of lp_types.h and the triangular crash on equality rows)."""
    rng = np.random.default_rng(seed)
    nnz_per_col = max(1, int(round(density * m)))
    starts = [0]
    rows, vals = [], []
    for c in range(n):
        k = max(1, min(m, rng.binomial(2 * nnz_per_col, 0.5)))
        r = np.sort(rng.choice(m, size=k, replace=False))
        v = rng.uniform(0.1, 1.0, size=k) * rng.choice([-1.0, 1.0], size=k)
        rows.extend(r.tolist())
        vals.extend(v.tolist())
        starts.append(len(rows))
    cs = np.asarray(starts, np.int64)
    ri = np.asarray(rows, np.int32)
    va = np.asarray(vals, np.float64)
    return _mixed_bounds_lp(rng, m, n, cs, ri, va, eq_frac, free_frac, boxed_frac, maximize,
                            f"sparse_{m}x{n}_s{seed}")


def _mixed_bounds_lp(rng, m, n, cs, ri, va, eq_frac, free_frac, boxed_frac, maximize, name):
    """Row/column bounds and costs of random_sparse_lp around a feasible
    point x0 (every bound type of lp_types.h), for the CSC (cs, ri, va)."""
    x0 = rng.uniform(0.0, 1.0, size=n)
    ax = np.zeros(m)
    for c in range(n):
        ax[ri[cs[c]:cs[c + 1]]] += va[cs[c]:cs[c + 1]] * x0[c]
    col_lb = np.zeros(n)
    col_ub = np.full(n, INF)
    kinds = rng.uniform(size=n)
    col_ub[kinds < boxed_frac] = 1.0 + rng.uniform(0, 2, size=(kinds < boxed_frac).sum())
    free = kinds > 1 - free_frac
    col_lb[free] = -INF
    col_ub[free] = INF
    row_lb = np.full(m, -INF)
    row_ub = ax + rng.uniform(0.0, 1.0, size=m)
    rk = rng.uniform(size=m)
    eq = rk < eq_frac
    row_lb[eq] = ax[eq]
    row_ub[eq] = ax[eq]
    ge = (rk >= eq_frac) & (rk < eq_frac + 0.3)
    row_lb[ge] = ax[ge] - rng.uniform(0.0, 1.0, size=ge.sum())
    row_ub[ge] = INF
    rng_rows = (rk >= eq_frac + 0.3) & (rk < eq_frac + 0.45)
    row_lb[rng_rows] = ax[rng_rows] - 1.0
    obj = rng.uniform(-1.0, 1.0, size=n)
    # Keep the LP bounded: free and unbounded-above columns get a cost that
    # a dense set of <= rows can bound only sometimes, so cap them by a box.
    unb = ~np.isfinite(col_ub)
    col_ub[unb] = 10.0 + rng.uniform(0, 5, size=unb.sum())
    col_lb[free] = -10.0 - rng.uniform(0, 5, size=free.sum())
    return LinearProgram(m, n, cs, ri, va, col_lb, col_ub, row_lb, row_ub, obj,
                         0.0, 1.0, maximize, name)


def staircase_lp(m, n, seed, block_rows=50, link_frac=0.2, eq_frac=0.1, free_frac=0.05,
                 boxed_frac=0.5, maximize=False):
    """Multi-period ("staircase") LP, the shape of Netlib's large models
    (scfxm, sctap, stocfor, pilot families): the rows form periods of about
    `block_rows` rows, each column has 2-7 non-zeros in its own period and,
    with probability `link_frac`, one in the next period (the carry-over of
    a multi-period model). The basis then factors with fill limited to the
    periods, as on the real models, instead of the dense fill of a uniformly
    random matrix. Bounds, row types and costs as in random_sparse_lp."""
    rng = np.random.default_rng(seed)
    periods = max(1, m // block_rows)
    edges = np.linspace(0, m, periods + 1).astype(np.int64)
    col_period = np.sort(rng.integers(0, periods, size=n))
    starts = [0]
    rows, vals = [], []
    for c in range(n):
        t = col_period[c]
        lo, hi = edges[t], edges[t + 1]
        k = int(min(hi - lo, rng.integers(2, 8)))
        r = rng.choice(np.arange(lo, hi), size=k, replace=False)
        if t + 1 < periods and rng.uniform() < link_frac:
            r = np.append(r, rng.integers(edges[t + 1], edges[t + 2]))
        r = np.sort(r)
        v = rng.uniform(0.1, 1.0, size=r.size) * rng.choice([-1.0, 1.0], size=r.size)
        rows.extend(r.tolist())
        vals.extend(v.tolist())
        starts.append(len(rows))
    cs = np.asarray(starts, np.int64)
    ri = np.asarray(rows, np.int32)
    va = np.asarray(vals, np.float64)
    return _mixed_bounds_lp(rng, m, n, cs, ri, va, eq_frac, free_frac, boxed_frac, maximize,
                            f"staircase_{m}x{n}_s{seed}")


def dual_phase1_lp(m, n, seed, density=0.05, unbounded_cols=0):
    """An LP whose slack basis is dual infeasible on unboxed columns, so that
    Glop's dual simplex from scratch runs its dedicated phase I
    (revised_simplex.cc:2198-2388) for many iterations: maximize c.x with c
    mostly > 0 over lower-bounded columns (x >= 0, no upper bound) with
    non-negative entries, upper-bounded columns (x <= u) with non-positive
    entries and c < 0, a few boxed and fixed columns, and <= / ranged rows
    with b > 0 (x = 0 is feasible, every improving ray meets a row).
    `unbounded_cols` trailing lower-bounded columns with a positive cost get
    no entries: the LP is then dual infeasible (phase I ends DUAL_INFEASIBLE)."""
    rng = np.random.default_rng(seed)
    nnz_per_col = max(1, int(round(density * m)))
    kinds = rng.uniform(size=n)  # < 0.6 lower, < 0.8 upper, < 0.95 boxed, else fixed
    starts = [0]
    rows, vals = [], []
    for c in range(n):
        if c >= n - unbounded_cols:
            starts.append(len(rows))
            continue
        k = max(1, min(m, rng.binomial(2 * nnz_per_col, 0.5)))
        r = np.sort(rng.choice(m, size=k, replace=False))
        v = rng.uniform(0.1, 1.0, size=k)
        if kinds[c] >= 0.6 and kinds[c] < 0.8:
            v = -v
        elif kinds[c] >= 0.8:
            v = v * rng.choice([-1.0, 1.0], size=k)
        rows.extend(r.tolist())
        vals.extend(v.tolist())
        starts.append(len(rows))
    cs = np.asarray(starts, np.int64)
    ri = np.asarray(rows, np.int32)
    va = np.asarray(vals, np.float64)
    col_lb = np.zeros(n)
    col_ub = np.full(n, INF)
    obj = rng.uniform(0.1, 1.0, size=n)
    upper = (kinds >= 0.6) & (kinds < 0.8)
    col_lb[upper] = -INF
    col_ub[upper] = rng.uniform(0.0, 1.0, size=upper.sum())
    obj[upper] = -obj[upper]
    boxed = (kinds >= 0.8) & (kinds < 0.95)
    col_ub[boxed] = 1.0 + rng.uniform(0, 2, size=boxed.sum())
    obj[boxed] *= rng.choice([-1.0, 1.0], size=boxed.sum())
    fixed = kinds >= 0.95
    col_ub[fixed] = 0.0
    if unbounded_cols:
        col_lb[n - unbounded_cols:] = 0.0
        col_ub[n - unbounded_cols:] = INF
        obj[n - unbounded_cols:] = rng.uniform(0.1, 1.0, size=unbounded_cols)
    # Row activity at x = 0 is the upper-bounded columns' contribution at
    # their bounds at most: b covers it.
    row_ub = rng.uniform(1.0, 2.0, size=m)
    row_lb = np.full(m, -INF)
    ranged = rng.uniform(size=m) < 0.2
    row_lb[ranged] = -1.0 - rng.uniform(0.0, 1.0, size=ranged.sum())
    return LinearProgram(m, n, cs, ri, va, col_lb, col_ub, row_lb, row_ub, obj,
                         0.0, 1.0, True, f"dual_phase1_{m}x{n}_s{seed}")


def fixed_order_matvec(At, x):
    """A @ x from the rows of At = A^T, summed column by column in index
    order with one rounding per multiply and per add. BLAS (`A @ x`) picks
    its kernel and thread split by CPU, so its last bits differ between this
    container and the GPU box: an LP built with it is not the same LP on both
    machines, and golden fixtures made here would not describe the LP the GPU
    test builds there."""
    acc = np.zeros(At.shape[1])
    for j in range(At.shape[0]):
        acc += At[j] * x[j]
    return acc


def dense_box_lp(m, n, seed, maximize=True):
    """Config 2 generator: A_ij ~ U(-1,1) dense,
    x0 ~ U(0,1), rows A x <= A x0 + U(0,1), 0 <= x <= 10, c ~ U(-1,1)."""
    rng = np.random.default_rng(seed)
    A = rng.uniform(-1.0, 1.0, size=(m, n))
    A[A == 0.0] = 0.5
    x0 = rng.uniform(0.0, 1.0, size=n)
    At = np.ascontiguousarray(A.T)
    del A
    rhs = fixed_order_matvec(At, x0) + rng.uniform(0.0, 1.0, size=m)
    cs = np.arange(0, (n + 1) * m, m, dtype=np.int64)
    ri = np.tile(np.arange(m, dtype=np.int32), n)
    va = At.reshape(-1)
    obj = rng.uniform(-1.0, 1.0, size=n)
    return LinearProgram(m, n, cs, ri, va, np.zeros(n), np.full(n, 10.0),
                         np.full(m, -INF), rhs, obj, 0.0, 1.0, maximize,
                         f"dense_{m}x{n}_s{seed}")


def sparse_c5_lp(m, n, per_col, seed):
    """Config 5 generator: about per_col non-zeros per
    column at distinct random rows, values U([-1,-0.1] u [0.1,1]),
    x0 ~ U(0,1), rows ranged [A x0 - s, A x0 + s] with s ~ U(0,1),
    0 <= x <= 10, c = A^T y0 + z with z >= 0 (minimize; dual-feasible-ish
    start). Vectorised so that m=1e5, n=1e6 builds in seconds."""
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, m, size=(n, per_col), dtype=np.int64)
    rows.sort(axis=1)
    keep = np.ones_like(rows, dtype=bool)
    keep[:, 1:] = rows[:, 1:] != rows[:, :-1]
    lens = keep.sum(axis=1)
    ri = rows[keep].astype(np.int32)
    nnz = ri.size
    mag = rng.uniform(0.1, 1.0, size=nnz)
    va = np.where(rng.random(nnz) < 0.5, -mag, mag)
    cs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=cs[1:])
    cols = np.repeat(np.arange(n, dtype=np.int64), lens)
    x0 = rng.uniform(0.0, 1.0, size=n)
    ax = np.bincount(ri, weights=va * x0[cols], minlength=m)
    slack = rng.uniform(0.0, 1.0, size=m)
    y0 = rng.uniform(-1.0, 1.0, size=m)
    aty = np.bincount(cols, weights=va * y0[ri], minlength=n)
    obj = aty + rng.uniform(0.0, 1.0, size=n)
    return LinearProgram(m, n, cs, ri, va, np.zeros(n), np.full(n, 10.0),
                         ax - slack, ax + slack, obj, 0.0, 1.0, False,
                         f"c5_{m}x{n}_s{seed}")


def from_dense_box(A, rng, maximize=True):
    """Box LP over an arbitrary (possibly partly sparse) matrix A: same row
    and bound construction as dense_box_lp, explicit zeros dropped."""
    m, n = A.shape
    x0 = rng.uniform(0.0, 1.0, size=n)
    rhs = fixed_order_matvec(np.ascontiguousarray(A.T), x0) + rng.uniform(0.0, 1.0, size=m)
    cols = [np.nonzero(A[:, j])[0] for j in range(n)]
    cs = np.zeros(n + 1, dtype=np.int64)
    cs[1:] = np.cumsum([len(c) for c in cols])
    ri = np.concatenate(cols).astype(np.int32) if n else np.zeros(0, np.int32)
    va = np.concatenate([A[c, j] for j, c in enumerate(cols)]) if n else np.zeros(0)
    obj = rng.uniform(-1.0, 1.0, size=n)
    return LinearProgram(m, n, cs, ri, va, np.zeros(n), np.full(n, 10.0),
                         np.full(m, -INF), rhs, obj, 0.0, 1.0, maximize,
                         f"mixed_{m}x{n}")


def to_scipy(lp):
    """Objective-only cross-check with scipy/HiGHS (test oracle pinning)."""
    import scipy.sparse as sp
    from scipy.optimize import linprog
    A = sp.csc_matrix((lp.vals, lp.row_idx, lp.col_starts), shape=(lp.m, lp.n))
    c = -lp.obj if lp.maximize else lp.obj
    A_ub, b_ub, A_eq, b_eq = [], [], [], []
    Ad = A.tocsr()
    for r in range(lp.m):
        lo, hi = lp.row_lb[r], lp.row_ub[r]
        row = Ad[r]
        if lo == hi:
            A_eq.append(row); b_eq.append(hi)
            continue
        if np.isfinite(hi):
            A_ub.append(row); b_ub.append(hi)
        if np.isfinite(lo):
            A_ub.append(-row); b_ub.append(-lo)
    res = linprog(c, A_ub=sp.vstack(A_ub) if A_ub else None, b_ub=b_ub or None,
                  A_eq=sp.vstack(A_eq) if A_eq else None, b_eq=b_eq or None,
                  bounds=list(zip(np.where(np.isfinite(lp.col_lb), lp.col_lb, None),
                                  np.where(np.isfinite(lp.col_ub), lp.col_ub, None))),
                  method="highs")
    if res.status != 0:
        return res.status, None
    val = res.fun + lp.obj_offset * (1 if not lp.maximize else -1)
    return 0, (-val if lp.maximize else val)


def presolve_lp(m, n, seed, maximize=False, tall=False):
    """Feasible LP around a point x0 carrying every structure Glop's presolve
    passes act on (glop/preprocessor.cc): fixed, empty, singleton and free
    doubleton columns, proportional columns and rows, empty, singleton,
    forcing and doubleton-equality rows, implied-free bounds, one-sided and
    free rows. tall=True makes rows >= 1.5 x columns (the dualizer's case)."""
    rng = np.random.default_rng(seed)
    if tall:
        m = max(m, int(1.8 * n))
    cols = []          # per column: dict row -> coeff
    x0 = []
    lb, ub, cost = [], [], []

    def add_col(entries, lo, hi, c, x):
        cols.append(dict(entries))
        lb.append(lo)
        ub.append(hi)
        cost.append(c)
        x0.append(x)
        return len(cols) - 1

    per_col = max(1, int(round(0.06 * m)))
    for _ in range(n):
        k = max(1, min(m, rng.binomial(2 * per_col, 0.5)))
        rows = rng.choice(m, size=k, replace=False)
        ent = {int(r): float(rng.uniform(0.2, 1.0) * rng.choice([-1.0, 1.0])) for r in rows}
        kind = rng.uniform()
        if kind < 0.55:
            lo, hi = 0.0, float(1.0 + rng.uniform(0, 2))
        elif kind < 0.75:
            lo, hi = 0.0, INF
        elif kind < 0.85:
            lo, hi = float(-rng.uniform(1, 3)), float(rng.uniform(1, 3))
        elif kind < 0.93:
            lo, hi = float(rng.uniform(0.5, 2.0)), float(rng.uniform(3.0, 5.0))  # shifted
        else:
            lo, hi = -INF, float(rng.uniform(1, 3))
        x = float(rng.uniform(max(lo, -1.0) if np.isfinite(lo) else -1.0,
                              min(hi, 3.0) if np.isfinite(hi) else 3.0))
        add_col(ent, lo, hi, float(rng.uniform(-1, 1)), x)
    base = len(cols)
    # fixed columns
    for _ in range(max(1, n // 20)):
        c = int(rng.integers(base))
        v = float(rng.uniform(-1, 2))
        add_col({int(r): float(rng.uniform(-1, 1)) for r in rng.choice(m, 3, replace=False)},
                v, v, float(rng.uniform(-1, 1)), v)
    # empty columns: cost pushes to a finite bound, or zero cost
    for k in range(3):
        c = [1.0, -1.0, 0.0][k]
        add_col({}, 0.0 if c >= 0 else -INF, 2.0 if c <= 0 else INF, c, 0.0)
    # proportional columns (copies of base columns, scaled), x0 = 0 in [.,.]
    for _ in range(max(1, n // 25)):
        src = int(rng.integers(base))
        f = float(rng.choice([-2.0, 0.5, 3.0]))
        same_cost = rng.uniform() < 0.6
        c = cost[src] * f if same_cost else float(rng.uniform(-1, 1))
        add_col({r: v * f for r, v in cols[src].items()}, 0.0, float(rng.uniform(1, 2)), c, 0.0)
    # singleton columns (slacks), some with cost
    for _ in range(max(1, n // 15)):
        r = int(rng.integers(m))
        add_col({r: float(rng.choice([-1.0, 1.0]) * rng.uniform(0.5, 2))}, 0.0,
                float(rng.choice([2.0, INF])), float(rng.choice([0.0, rng.uniform(-1, 1)])), 0.0)
    # free doubleton columns, zero cost
    for _ in range(2):
        r1, r2 = (int(v) for v in rng.choice(m, 2, replace=False))
        add_col({r1: float(rng.uniform(0.5, 1.5)), r2: float(-rng.uniform(0.5, 1.5))},
                -INF, INF, 0.0, float(rng.uniform(-1, 1)))
    nrows = m
    extra_rows = []    # (entries dict col -> coeff, kind)
    # doubleton equality rows
    for _ in range(max(1, m // 15)):
        i, j = (int(v) for v in rng.choice(base, 2, replace=False))
        extra_rows.append(({i: float(rng.uniform(0.5, 2)), j: float(-rng.uniform(0.5, 2))}, "eq"))
    # singleton rows (tighten a variable)
    for _ in range(max(1, m // 20)):
        c = int(rng.integers(base))
        extra_rows.append(({c: float(rng.choice([-1.0, 1.0]) * rng.uniform(0.5, 2))}, "rng"))
    # forcing row: positive coefficients on boxed columns at their upper bound
    boxed = [c for c in range(base) if lb[c] == 0.0 and np.isfinite(ub[c])]
    if len(boxed) >= 3:
        pick = [int(v) for v in rng.choice(boxed, 3, replace=False)]
        for c in pick:
            x0[c] = ub[c]
        extra_rows.append(({c: float(rng.uniform(0.5, 1.5)) for c in pick}, "forcing"))
    # proportional rows: scaled copies of the first rows (their entries)
    col_rows = [dict() for _ in range(m)]
    for c, ent in enumerate(cols):
        for r, v in ent.items():
            col_rows[r][c] = v
    for r in range(min(3, m)):
        if col_rows[r]:
            f = float(rng.choice([-1.5, 2.0]))
            extra_rows.append(({c: v * f for c, v in col_rows[r].items()}, "any"))
    extra_rows.append(({}, "empty"))
    for ent, kind in extra_rows:
        for c, v in ent.items():
            cols[c][nrows] = v
        nrows += 1
    ncols = len(cols)
    x0 = np.asarray(x0)
    ax = np.zeros(nrows)
    for c, ent in enumerate(cols):
        for r, v in ent.items():
            ax[r] += v * x0[c]
    row_lb = np.full(nrows, -INF)
    row_ub = np.full(nrows, INF)
    kinds = [None] * m + [k for _, k in extra_rows]
    for r in range(nrows):
        k = kinds[r]
        u = rng.uniform()
        if k == "eq" or (k is None and u < 0.2):
            row_lb[r] = row_ub[r] = ax[r]
        elif k == "forcing":
            row_lb[r] = ax[r]
        elif k == "empty":
            row_lb[r], row_ub[r] = -1.0, 1.0
        elif k == "rng" or u < 0.35:
            row_lb[r], row_ub[r] = ax[r] - rng.uniform(0, 1), ax[r] + rng.uniform(0, 1)
        elif u < 0.65:
            row_ub[r] = ax[r] + rng.uniform(0, 1)
        elif u < 0.97:
            row_lb[r] = ax[r] - rng.uniform(0, 1)
        # else free row
    cs = [0]
    ri, va = [], []
    for ent in cols:
        for r in sorted(ent):
            ri.append(r)
            va.append(ent[r])
        cs.append(len(ri))
    # keep bounded: cap infinite sides that the cost pushes towards
    col_lb = np.asarray(lb, float)
    col_ub = np.asarray(ub, float)
    obj = np.asarray(cost, float)
    sgn = -1.0 if maximize else 1.0
    push_up = sgn * obj < 0
    cap = ~np.isfinite(col_ub) & push_up
    col_ub[cap] = 20.0
    push_dn = sgn * obj > 0
    capl = ~np.isfinite(col_lb) & push_dn
    col_lb[capl] = -20.0
    return LinearProgram(nrows, ncols, np.asarray(cs, np.int64), np.asarray(ri, np.int32),
                         np.asarray(va, float), col_lb, col_ub, row_lb, row_ub, obj, 0.5, 1.0,
                         maximize, f"presolve_{nrows}x{ncols}_s{seed}")


def tiny_mixed_lp(rng, max_dim=7):
    """Small integer-coefficient LP with every bound type (free, one-sided,
    boxed, fixed, crossing-free), sometimes a duplicated column and row; about
    a third end optimal, the rest infeasible or unbounded (presolve fuzzing)."""
    m = int(rng.integers(1, max_dim))
    n = int(rng.integers(1, max_dim + 1))
    a = rng.integers(-3, 4, size=(m, n)).astype(float) * (rng.uniform(size=(m, n)) < 0.5)
    if rng.uniform() < 0.3:
        if n > 1:
            a[:, n - 1] = a[:, 0] * rng.choice([-2.0, 0.5, 1.0])
        if m > 1:
            a[m - 1, :] = a[0, :] * rng.choice([-1.0, 2.0])

    def bounds(k):
        lb, ub = np.zeros(k), np.zeros(k)
        for i in range(k):
            lo = float(rng.integers(-3, 4))
            hi = lo + float(rng.integers(0, 4))
            lb[i], ub[i] = [(lo, hi), (-INF, hi), (lo, INF), (-INF, INF), (lo, lo),
                            (lo, hi)][int(rng.integers(6))]
        return lb, ub

    clb, cub = bounds(n)
    rlb, rub = bounds(m)
    obj = rng.integers(-3, 4, size=n).astype(float)
    return LinearProgram.from_dense(a, clb, cub, rlb, rub, obj, float(rng.integers(-2, 3)),
                                    maximize=bool(rng.integers(2)))
