"""RCCL bound sharing behind the C ABI (include/mi_lp.h mi_lp_comm_*,
mi_lp_share_bound; engine/comm.hip), called through ctypes as a C++ CP-SAT
host would bind it: the all-reduce(min/max) of one float64 over the ranks
that SharedResponseManager::UpdateInnerObjectiveBounds stands for across
GPUs (sat/synchronization.h:306).

One-GPU box: a one-rank communicator (RCCL refuses two ranks on one GPU);
with two or more GPUs, two processes, one GPU each."""
import ctypes
import math
import multiprocessing as mproc

import numpy as np
import pytest

from mi_glop import distributed, engine

pytestmark = pytest.mark.gpu


def test_one_rank_share_bound_and_device_collectives():
    c = distributed.NativeComm(0, 1, 0)
    assert (c.rank(), c.size()) == (0, 1)
    for v in (3.25, -math.inf, math.inf, -0.0, 1e300):
        assert c.share_bound(v) == v
        assert c.share_bound(v, distributed.NativeComm.MAX) == v
    L = engine.lib()
    import torch
    x = torch.arange(8, dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    assert L.mi_lp_comm_allreduce_device(c._h, ctypes.c_void_p(x.data_ptr()), 8, 0) == 0
    np.testing.assert_array_equal(x.cpu().numpy(), np.arange(8.0))
    y = torch.empty(8, dtype=torch.float64, device="cuda:0")
    assert L.mi_lp_comm_allgather_device(c._h, ctypes.c_void_p(x.data_ptr()),
                                         ctypes.c_void_p(y.data_ptr()), 64) == 0
    np.testing.assert_array_equal(y.cpu().numpy(), np.arange(8.0))
    # Argument errors come back as codes, not crashes.
    assert L.mi_lp_share_bound(c._h, None, 0) != 0
    v = ctypes.c_double(1.0)
    assert L.mi_lp_share_bound(c._h, ctypes.byref(v), 7) != 0
    c.close()


def _rank(rank, world, uid, values, q):
    try:
        c = distributed.NativeComm(rank, world, rank, uid=uid)
        lo = c.share_bound(values[rank], distributed.NativeComm.MIN)
        hi = c.share_bound(values[rank], distributed.NativeComm.MAX)
        c.close()
        q.put((rank, lo, hi))
    except Exception as e:  # reported to the parent
        q.put((rank, repr(e), None))


@pytest.mark.skipif(engine.device_count() < 2, reason="RCCL needs one GPU per rank")
def test_two_ranks_share_bound():
    uid = distributed.NativeComm.unique_id()
    values = [7.5, -2.25]
    ctx = mproc.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, 2, uid, values, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert [g[1:] for g in got] == [(min(values), max(values))] * 2, got
