"""World-size-2 gloo test of the multi-GPU layer (mi_glop.distributed) on
CPU: the node's children are sharded across ranks, each rank solves its
shard (the CPU oracle stands in for the GPU engine here), and the RCCL
all-reduce(min) of the bound -- gloo on CPU -- must equal the single-process
minimum over all children; the MAX-over-ranks timing helper likewise."""
import math
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _children():
    import jobshop
    from mi_glop import abi
    import oracle_lib
    lp, ycols = jobshop.relaxation(jobshop.FT06)
    root = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=1))
    root.load(lp)
    root.solve()
    lbs, ubs = jobshop.child_bounds(lp, ycols, 10, 3)
    return lp, root.state(), lbs, ubs


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "or-tools_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mi_glop import abi, distributed
    import oracle_lib
    lp, state, lbs, ubs = _children()
    b, e = distributed.shard(len(lbs), rank, world)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    ws = [oracle_lib.OracleLp(p) for _ in range(2)]
    for w in ws:
        w.load(lp)
    res = oracle_lib.batch_solve_bounds(ws, lbs[b:e], ubs[b:e], state)
    local = distributed.best_bound(res, abi.OPTIMAL)
    shared = distributed.share_bound(local, dist)
    slowest = distributed.max_over_ranks(float(rank + 1), dist)
    total = distributed.sum_over_ranks(e - b, dist)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(f"{b} {e} {local!r} {shared!r} {slowest!r} {total!r}\n")
    dist.destroy_process_group()


def test_shard_partition():
    from mi_glop import distributed
    for count in (0, 1, 7, 16, 1001):
        for world in (1, 2, 3, 8):
            blocks = [distributed.shard(count, r, world) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == count
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(world - 1))
            sizes = [e - b for b, e in blocks]
            assert max(sizes) - min(sizes) <= 1


def test_lpt_partition():
    from mi_glop import distributed
    costs = [5.0, 1.0, 7.0, 3.0, 3.0, 2.0, 9.0, 4.0]
    for world in (1, 2, 3, 8):
        parts = distributed.lpt_partition(costs, world)
        assert sorted(i for p in parts for i in p) == list(range(len(costs)))
        loads = [sum(costs[i] for i in p) for p in parts]
        # LPT bound: makespan <= 4/3 of the optimum; the optimum >= both
        # the average load and the largest job.
        assert max(loads) <= 4.0 / 3.0 * max(sum(costs) / world, max(costs)) + 1e-9
    assert distributed.lpt_partition(costs, 2) == [[1, 4, 6, 7], [0, 2, 3, 5]]  # 17 + 17
    import netlib_suite
    suite = netlib_suite.suite(max_rows=200)
    parts = distributed.lpt_partition([distributed.lp_cost(lp) for lp in suite], 4)
    assert sum(len(p) for p in parts) == len(suite)


def test_bound_share_world2(tmp_path):
    from mi_glop import abi, distributed
    import oracle_lib
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    rows = [open(tmp_path / f"r{r}.txt").read().split() for r in range(2)]
    # Single-process reference over all children.
    lp, state, lbs, ubs = _children()
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    best = math.inf
    for i in range(len(lbs)):
        o.set_variable_bounds(lbs[i], ubs[i])
        o.load_basis_state(state)
        r = o.solve()
        if r.problem_status == abi.OPTIMAL:
            best = min(best, r.objective)
    assert [int(rows[0][0]), int(rows[0][1]), int(rows[1][0]), int(rows[1][1])] == [0, 5, 5, 10]
    for row in rows:
        assert float(row[3]) == best  # all-reduce(min) = global best bound
        assert float(row[4]) == 2.0   # max over ranks
        assert float(row[5]) == 10.0  # sum over ranks: every child counted once
    assert min(float(rows[0][2]), float(rows[1][2])) == best


# --- single-LP column split: the exchange step ------

def _split_problem():
    """A config-5-shaped LP's [A | I] CSC, a rho, reduced costs: the inputs of
    one dual ratio test (entering_variable.cc:37-130)."""
    import numpy as np
    import lp_gen
    lp = lp_gen.sparse_c5_lp(300, 3000, 6, 123)
    m, n = lp.m, lp.n
    starts = np.concatenate([lp.col_starts, lp.col_starts[-1] + 1 + np.arange(m)])
    rows = np.concatenate([lp.row_idx, np.arange(m)])
    vals = np.concatenate([lp.vals, np.ones(m)])
    rng = np.random.default_rng(7)
    rho = rng.uniform(-1, 1, m) * (rng.random(m) < 0.2)
    rc = np.abs(rng.normal(size=n + m))
    return starts, rows, vals, rho, rc


def _alpha(starts, rows, vals, rho, b, e):
    import numpy as np
    return np.array([float(np.dot(rho[rows[starts[c]:starts[c + 1]]],
                                  vals[starts[c]:starts[c + 1]])) for c in range(b, e)])


def _local_filter(alpha, rc, b, tol=1e-9):
    """Harris bound of the block (min over its breakpoints of (|rc|+tol)/|alpha|)
    and its breakpoints, as (column, alpha, ratio)."""
    import numpy as np
    nz = np.abs(alpha) > 1e-9
    ratio = np.where(nz, rc / np.where(nz, np.abs(alpha), 1.0), np.inf)
    harris = np.where(nz, (rc + tol) / np.where(nz, np.abs(alpha), 1.0), np.inf)
    return float(harris.min()), [(b + i, float(alpha[i]), float(ratio[i]))
                                 for i in range(len(alpha)) if nz[i]]


def _split_worker(rank, world, port, out_dir):
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "or-tools_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mi_glop import distributed
    starts, rows, vals, rho, rc = _split_problem()
    bounds = distributed.column_blocks(starts, world)
    b, e = bounds[rank], bounds[rank + 1]
    bound, cands = _local_filter(_alpha(starts, rows, vals, rho, b, e), rc[b:e], b)
    bound = distributed.min_bound(bound, dist)           # all-reduce(min)
    keep = [(c, a) for c, a, r in cands if r <= bound * (1.0 + 1e-9)]
    cols, coeffs = distributed.gather_candidates([c for c, _ in keep], [a for _, a in keep], dist)
    q = cols[0] if cols else 0
    owner = distributed.owner_of(q, bounds)
    col = [0.0] * len(rho)
    if owner == rank:
        for k in range(starts[q], starts[q + 1]):
            col[rows[k]] = float(vals[k])
    col = distributed.broadcast_column(col, owner, dist)  # a_q from its owner
    with open(os.path.join(out_dir, f"s{rank}.txt"), "w") as f:
        f.write(repr((b, e, bound, cols, coeffs, q, col)) + "\n")
    dist.destroy_process_group()


def test_column_blocks_match_engine_rule():
    import numpy as np
    from mi_glop import distributed
    starts = np.concatenate([[0], np.cumsum(np.random.default_rng(3).integers(1, 12, 5000))])
    for world in (1, 2, 3, 8):
        bd = distributed.column_blocks(starts, world)
        assert bd[0] == 0 and bd[-1] == 5000 and bd == sorted(bd)
        assert all(x % 64 == 0 for x in bd[1:-1])
        assert distributed.owner_of(bd[-2], bd) == world - 1 or bd[-2] == bd[-1]


def test_column_split_exchange_world2(tmp_path):
    """Two ranks each own a column block; after all-reduce(min) of the bound,
    all-gather of the candidates and broadcast of a_q, every rank holds
    exactly what the single-process join computes (the virtual-shard join of
    engine/device_shards.hip, which the GPU tests pin to the oracle)."""
    from mi_glop import distributed
    port = _free_port()
    mp.start_processes(_split_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    import ast
    got = [ast.literal_eval(open(tmp_path / f"s{r}.txt").read()) for r in range(2)]
    starts, rows, vals, rho, rc = _split_problem()
    n_total = len(starts) - 1
    bound, cands = _local_filter(_alpha(starts, rows, vals, rho, 0, n_total), rc, 0)
    keep = [(c, a) for c, a, r in cands if r <= bound * (1.0 + 1e-9)]
    assert got[0][1] == got[1][0]  # contiguous blocks
    for g in got:
        assert g[2] == bound
        assert g[3] == [c for c, _ in keep] and g[4] == [a for _, a in keep]
    q = keep[0][0]
    ref = [0.0] * len(rho)
    for k in range(starts[q], starts[q + 1]):
        ref[rows[k]] = float(vals[k])
    assert got[0][6] == ref and got[1][6] == ref and got[0][5] == q
