"""The split's same-node exchange (engine/exchange.cc, mi_exchange_*): an
all-gather of host bytes through POSIX shared memory, in C++. It needs no
GPU, so it runs here with real processes: every rank must receive every
rank's bytes in rank order, for empty, small and multi-round (longer than a
slot) messages, many calls in a row (the two-bank reuse), and nothing may be
left in /dev/shm."""
import multiprocessing as mp
import os
import uuid

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _payload(call, rank):
    rng = np.random.default_rng(1000 * call + rank)
    n = int(rng.choice([0, 1, 7, 100, 4096, 4097, 20000]))
    return rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()


def _worker(name, rank, world, calls, q):
    import sys
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "or-tools_amd")]
    from mi_glop import engine
    try:
        x = engine.ShmExchange(name, rank, world, slot_bytes=4096)
        ok = True
        for c in range(calls):
            mine = _payload(c, rank)
            sizes = [len(_payload(c, r)) for r in range(world)]
            got = x.allgather(mine, sizes)
            want = b"".join(_payload(c, r) for r in range(world))
            ok = ok and got == want
        x.close()
        q.put((rank, ok))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def _run(world, calls=60):
    name = f"/mi_lp_test_{uuid.uuid4().hex}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(name, r, world, calls, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(v is True for v in res.values()), res
    assert not os.path.exists("/dev/shm" + name), "segment left behind"


def test_exchange_two_ranks():
    _run(2)


def test_exchange_five_ranks():
    _run(5, calls=30)


def test_exchange_single_rank():
    _run(1, calls=5)
