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


# --- single-LP column split: the engine's exchange ---

def _split_worker(rank, world, port, out_dir):
    """Drives the engine's exchange callback (mi_lp_allgather_fn, built by
    engine.allgather_callback over distributed.allgather_bytes) the way
    DeviceLp::ExchangeParts does: sizes first (8 bytes per rank), then the
    variable-size block messages, including an empty one."""
    import ctypes
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "or-tools_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mi_glop import distributed, engine
    cb = engine.allgather_callback(world, lambda d, s: distributed.allgather_bytes(d, s, dist))
    got = []
    for msg in (b"", bytes(range(7)) * (rank + 1), bytes([rank]) * (1000 * rank)):
        n = ctypes.c_int64(len(msg))
        sizes = (ctypes.c_int64 * world)()
        eight = (ctypes.c_int64 * world)(*([8] * world))
        assert cb(None, ctypes.byref(n), 8, sizes, eight) == 0
        total = sum(sizes)
        recv = ctypes.create_string_buffer(max(1, total))
        send = ctypes.create_string_buffer(msg, max(1, len(msg)))
        assert cb(None, send, len(msg), recv, sizes) == 0
        got.append((list(sizes), recv.raw[:total].hex()))
    # A failing all-gather reports 1 instead of raising through the C ABI.
    bad = engine.allgather_callback(world, lambda d, s: b"short")
    n = ctypes.c_int64(3)
    sizes = (ctypes.c_int64 * world)(3, 3)
    recv = ctypes.create_string_buffer(6)
    got.append(bad(None, ctypes.byref(n), 3, recv, sizes))
    with open(os.path.join(out_dir, f"s{rank}.txt"), "w") as f:
        f.write(repr(got) + "\n")
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
    """The byte all-gather the engine's column split calls (gloo, world 2):
    every rank receives every rank's message in rank order, sizes included,
    for empty and unequal messages; a broken collective returns an error
    code. (The engine split itself needs a GPU: tests/test_split_gpu.py runs
    it across two processes against the unsplit engine and the oracle.)"""
    port = _free_port()
    mp.start_processes(_split_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    import ast
    got = [ast.literal_eval(open(tmp_path / f"s{r}.txt").read()) for r in range(2)]
    msgs = [[b"", bytes(range(7)) * (r + 1), bytes([r]) * (1000 * r)] for r in range(2)]
    for g in got:
        for k in range(3):
            sizes, data = g[k]
            assert sizes == [len(msgs[0][k]), len(msgs[1][k])]
            assert bytes.fromhex(data) == msgs[0][k] + msgs[1][k]
        assert g[3] == 1
