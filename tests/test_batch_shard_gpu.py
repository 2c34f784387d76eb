"""Batched LPs sharded across two processes with the ENGINE solving
(SURVEY 8(e), configs 3 and 4): each process owns its shard of one search
node's branch LPs (both branches of a variable on one rank, as bench.py's
config-4 section cuts them) or its LPT share of a Netlib-shaped suite
(config 3), solves it through the engine's batch APIs on the one GPU of the
box, and the ranks share the node bound with an all-reduce (gloo here: RCCL
refuses two ranks on one GPU; bench.py uses RCCL with one GPU per rank).
Every child's status, iteration count and objective must equal the oracle's,
and the shared bound must equal the single-process fold over all children
(the property SharedResponseManager::UpdateInnerObjectiveBounds relies on,
sat/synchronization.h:306)."""
import ast
import math
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _node():
    """The search node: job-shop relaxation, its root solve by the oracle
    (the warm-start state and the fractional point), and the BranchOnVar
    children of its most fractional order variables."""
    import jobshop
    import oracle_lib
    from mi_glop import abi, cpsat
    jobs = jobshop.random_instance(8, 5, 20261015)
    lp, ycols = jobshop.relaxation(jobs)
    root = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=1))
    root.load(lp)
    rr = root.solve()
    x = root.primal()
    node = cpsat.IntegerTrail(lp.col_lb, lp.col_ub,
                              obj_lb=math.ceil(rr.objective - cpsat.K_CP_EPSILON))
    cols = cpsat.fractional_columns(x, ycols, limit=24)
    return lp, root.state(), node, x, cols


def _row(r):
    return (int(r.problem_status), int(r.error_code), int(r.iterations), float(r.objective).hex())


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "or-tools_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mi_glop import abi, cpsat, distributed, engine
    import netlib_suite
    # Config 4: this rank's block of the node's branching variables.
    lp, state, node, x, cols_all = _node()
    b, e = distributed.shard(len(cols_all), rank, world)
    lbs, ubs = cpsat.branch_lps(node, x, cols_all[b:e])
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    workers = [engine.LpHandle(p) for _ in range(8)]
    for w in workers:
        w.load(lp)
    res = engine.batch_solve_bounds(workers, lbs, ubs, state)
    local = distributed.best_bound(res, abi.OPTIMAL)
    shared = distributed.share_bound(local, dist)
    # Config 3: this rank's LPT share of the suite.
    suite = netlib_suite.suite(max_rows=300)
    mine = distributed.lpt_partition([distributed.lp_cost(q) for q in suite], world)[rank]
    handles = []
    for i in mine:
        h = engine.LpHandle(abi.default_params())
        h.load(suite[i])
        handles.append(h)
    res3 = engine.batch_solve(handles, num_threads=4)
    out = {"block": [b, e], "children": [_row(r) for r in res], "local": float(local).hex(),
           "shared": float(shared).hex(), "c3": {i: _row(r) for i, r in zip(mine, res3)}}
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(repr(out) + "\n")
    for h in workers + handles:
        h.close()
    dist.destroy_process_group()


def test_engine_batches_sharded_across_processes(tmp_path):
    from mi_glop import abi, cpsat
    import netlib_suite
    import oracle_lib
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    got = [ast.literal_eval(open(tmp_path / f"r{r}.txt").read()) for r in range(2)]
    # Single-process reference: the oracle over every child, in order.
    lp, state, node, x, cols = _node()
    lbs, ubs = cpsat.branch_lps(node, x, cols)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    ref, best = [], math.inf
    for i in range(len(lbs)):
        o.set_variable_bounds(lbs[i], ubs[i])
        o.load_basis_state(state)
        r = o.solve()
        ref.append(_row(r))
        if r.problem_status == abi.OPTIMAL:
            best = min(best, r.objective)
    assert got[0]["block"][0] == 0 and got[0]["block"][1] == got[1]["block"][0]
    assert got[1]["block"][1] == len(cols)
    assert got[0]["children"] + got[1]["children"] == ref
    for g in got:
        assert float.fromhex(g["shared"]) == best  # all-reduce(min) = the global bound
    assert min(float.fromhex(g["local"]) for g in got) == best
    suite = netlib_suite.suite(max_rows=300)
    c3 = {**got[0]["c3"], **got[1]["c3"]}
    assert sorted(c3) == list(range(len(suite)))  # every LP on exactly one rank
    assert not set(got[0]["c3"]) & set(got[1]["c3"])
    for i, q in enumerate(suite):
        oq = oracle_lib.OracleLp(abi.default_params())
        oq.load(q)
        assert c3[i] == _row(oq.solve()), i
