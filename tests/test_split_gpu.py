"""One LP split across two processes (the single-LP column
split, mi_lp_set_exchange). Each process runs the engine on the same GPU with
its own column block of [A | I]; the blocks' results are joined through the
engine's C++ shared-memory all-gather (engine/exchange.cc, the default) or a
gloo all-gather (mi_glop.distributed.attach_column_split). Both processes
must end with exactly the unsplit engine's and the oracle's solve: status,
iterations, basis, statuses and values bit for bit (the reference pins the
same property for its sharder, pdlp/sharder_test.cc:128-172)."""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _lp(case):
    import lp_gen
    if case == "sparse_dual":
        return lp_gen.sparse_c5_lp(1500, 15000, 8, 91), 1
    if case == "sparse_primal":
        return lp_gen.random_sparse_lp(300, 2000, 0.02, 92), 0
    return lp_gen.dense_box_lp(120, 900, 93), 0


def _digest(h, r):
    var, cons = h.statuses()
    parts = [h.basis(), h.state(), var, cons, h.primal(), h.duals(), h.reduced_costs()]
    return (int(r.problem_status), int(r.error_code), int(r.iterations), float(r.objective).hex(),
            hashlib.sha256(b"".join(np.ascontiguousarray(p).tobytes() for p in parts)).hexdigest())


def _worker(rank, world, port, case, env, out_dir, transport):
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "or-tools_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **env)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mi_glop import abi, distributed, engine
    lp, dual = _lp(case)
    h = engine.LpHandle(abi.default_params(use_dual_simplex=dual, max_number_of_iterations=4000))
    _, _, xchg = distributed.attach_column_split(h, dist, transport=transport)
    h.load(lp)
    r = h.solve()
    out = _digest(h, r)
    ex = h.kernel_stats()["exchange"]
    assert ex["launches"] > 0, "the joins did not go through the exchange"
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(repr(out) + "\n")
    h.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,env,transport", [
    ("sparse_dual", {}, "shm"),
    ("sparse_dual", {"MILP_DEVICE_DUAL": "force"}, "shm"),
    ("sparse_primal", {}, "shm"),
    ("dense_primal", {}, "shm"),
    ("sparse_dual", {}, "gloo"),
], ids=["dual", "dual_device_mode", "primal_sparse", "primal_dense", "dual_gloo"])
def test_column_split_across_processes(case, env, transport, tmp_path, monkeypatch):
    import ast
    from mi_glop import abi, engine
    import parity_util
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, case, env, str(tmp_path), transport), nprocs=2,
                       join=True,
                       start_method="spawn")
    got = [ast.literal_eval(open(tmp_path / f"r{r}.txt").read()) for r in range(2)]
    lp, dual = _lp(case)
    p = abi.default_params(use_dual_simplex=dual, max_number_of_iterations=4000)
    o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q))
    parity_util.compare(o, ro, g, rg, lp)
    ref = _digest(g, rg)
    assert got[0] == ref and got[1] == ref, (got, ref)
