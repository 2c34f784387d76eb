"""Config 4 workload: LP relaxations of a disjunctive
job-shop model, as CP-SAT's LP call-out sees them during search.

Model (big-M disjunctive MIP, LP-relaxed): start times s_o >= 0 per
operation, makespan C; precedence rows s_{j,k+1} - s_{j,k} >= d_{j,k};
makespan rows C - s_{j,last} >= d_{j,last}; for each pair (a, b) of
operations on one machine an order variable y_ab in [0, 1] with
  s_a + d_a - s_b - M y_ab <= 0   and   s_b + d_b - s_a + M y_ab <= M.
Minimize C. A search node emits many child LPs that share the matrix and
differ by one or two branched y bounds (mirrors BranchOnVar,
linear_programming_constraint.cc:485-584); they are solved with the dual
simplex warm-started from the parent basis (LoadStateForNextSolve).

ft06 is the reference's own instance (ortools/scheduling/testdata/ft06,
Fisher & Thompson 6x6; machine/duration pairs per job copied as data).
The 50x10 instance is seeded random (durations U[1, 99]) in the shape of
ta041 (50_10_01_ta041.txt)."""
import itertools

import numpy as np

from mi_glop.lp import INF, LinearProgram

# ortools/scheduling/testdata/ft06: per job, (machine, duration) in order.
FT06 = [
    [(2, 1), (0, 3), (1, 6), (3, 7), (5, 3), (4, 6)],
    [(1, 8), (2, 5), (4, 10), (5, 10), (0, 10), (3, 4)],
    [(2, 5), (3, 4), (5, 8), (0, 9), (1, 1), (4, 7)],
    [(1, 5), (0, 5), (2, 5), (3, 3), (4, 8), (5, 9)],
    [(2, 9), (1, 3), (4, 5), (5, 4), (0, 3), (3, 1)],
    [(1, 3), (3, 3), (5, 9), (0, 10), (4, 4), (2, 1)],
]


def random_instance(num_jobs, num_machines, seed):
    rng = np.random.default_rng(seed)
    jobs = []
    for _ in range(num_jobs):
        order = rng.permutation(num_machines)
        dur = rng.integers(1, 100, size=num_machines)
        jobs.append([(int(m), int(d)) for m, d in zip(order, dur)])
    return jobs


def relaxation(jobs):
    """Returns (LinearProgram, y_columns) of the big-M LP relaxation."""
    ops = [(j, k, m, d) for j, job in enumerate(jobs) for k, (m, d) in enumerate(job)]
    op_id = {(j, k): i for i, (j, k, _, _) in enumerate(ops)}
    n_ops = len(ops)
    big_m = float(sum(d for (_, _, _, d) in ops))
    by_machine = {}
    for i, (_, _, m, _) in enumerate(ops):
        by_machine.setdefault(m, []).append(i)
    pairs = [p for m in sorted(by_machine) for p in itertools.combinations(by_machine[m], 2)]
    c_col = n_ops + len(pairs)
    n = c_col + 1
    cols = [[] for _ in range(n)]  # (row, value)
    row_lb, row_ub = [], []

    def add_row(entries, lo, hi):
        r = len(row_lb)
        for c, v in entries:
            cols[c].append((r, v))
        row_lb.append(lo)
        row_ub.append(hi)

    for j, job in enumerate(jobs):
        for k in range(len(job) - 1):
            a, b = op_id[(j, k)], op_id[(j, k + 1)]
            add_row([(b, 1.0), (a, -1.0)], float(job[k][1]), INF)
        last = op_id[(j, len(job) - 1)]
        add_row([(c_col, 1.0), (last, -1.0)], float(job[-1][1]), INF)
    for p, (a, b) in enumerate(pairs):
        y = n_ops + p
        da, db = float(ops[a][3]), float(ops[b][3])
        add_row([(a, 1.0), (b, -1.0), (y, -big_m)], -INF, -da)
        add_row([(a, -1.0), (b, 1.0), (y, big_m)], -INF, big_m - db)
    starts = np.zeros(n + 1, dtype=np.int64)
    rows, vals = [], []
    for c in range(n):
        for r, v in sorted(cols[c]):
            rows.append(r)
            vals.append(v)
        starts[c + 1] = len(rows)
    m = len(row_lb)
    col_lb = np.zeros(n)
    col_ub = np.full(n, INF)
    col_ub[n_ops:c_col] = 1.0
    obj = np.zeros(n)
    obj[c_col] = 1.0
    lp = LinearProgram(m, n, starts, np.array(rows, dtype=np.int32), np.array(vals),
                       col_lb, col_ub, np.array(row_lb), np.array(row_ub), obj, 0.0, 1.0,
                       False, f"jobshop_{len(jobs)}x{len(jobs[0])}")
    return lp, np.arange(n_ops, c_col)


def child_bounds(lp, y_cols, count, seed, branched=2):
    """count (col_lb, col_ub) pairs: each fixes `branched` random order
    variables to 0 or 1 (one search node's children)."""
    rng = np.random.default_rng(seed)
    lbs = np.repeat(lp.col_lb[None, :], count, axis=0)
    ubs = np.repeat(lp.col_ub[None, :], count, axis=0)
    for i in range(count):
        picks = rng.choice(y_cols, size=branched, replace=False)
        for c in picks:
            v = float(rng.integers(0, 2))
            lbs[i, c] = v
            ubs[i, c] = v
    return lbs, ubs
