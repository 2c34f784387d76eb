"""Multi-GPU layer for batched LP relaxations.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).
Independent LPs shard with no data-path collective. The only exchange is
all-reduce(min) of the best bound after each round of children, the
cross-GPU analogue of SharedResponseManager::UpdateInnerObjectiveBounds
(sat/synchronization.h:306). It is an 8-byte message, latency-bound over
xGMI.
"""
import math


def shard(count, rank, world):
    """Contiguous block [begin, end) of `count` LPs owned by `rank`. The
    blocks differ in size by at most one."""
    base, extra = divmod(count, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def lpt_partition(costs, world):
    """Longest-processing-time-first assignment of independent LPs to ranks
    (SURVEY.md 8(e)): LPs in decreasing cost order, each to the rank with the
    smallest load so far (ties: lowest rank). Deterministic, so every rank
    computes the same partition without a collective. Returns one index list
    per rank, each in increasing LP index order."""
    loads = [0.0] * world
    parts = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        r = min(range(world), key=lambda q: (loads[q], q))
        loads[r] += costs[i]
        parts[r].append(i)
    return [sorted(p) for p in parts]


def lp_cost(lp):
    """LPT weight of one LP: non-zeros x rows (work per iteration x a
    row-proportional iteration count)."""
    return float(lp.nnz + lp.m) * float(lp.m)


def best_bound(results, optimal_status=0):
    """Minimum objective over the children that reached OPTIMAL (inf if none)."""
    vals = [r.objective for r in results if r.problem_status == optimal_status]
    return min(vals) if vals else math.inf


def share_bound(best, dist=None, device=None):
    """All-reduce(min) of a rank's best bound. It is a no-op without a
    process group. `device` is "cuda" for RCCL and None/"cpu" for gloo."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return best
    import torch
    t = torch.tensor([best], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


class NativeComm:
    """The engine's RCCL communicator (mi_lp_comm_*, engine/comm.hip): the
    C-ABI path a C++ CP-SAT host uses to share its bound across GPUs
    (sat/synchronization.h:306) without Python. Here the unique id travels
    over an existing process group (any backend); the all-reduce itself is
    ncclAllReduce(ncclFloat64, min/max) on the engine's device buffer."""

    MIN, MAX = 0, 1

    def __init__(self, rank, world, device, uid=None, dist=None):
        import ctypes
        from . import engine
        self._L = L = engine.lib()
        if uid is None:
            buf = (ctypes.c_uint8 * 128)()
            if rank == 0 and L.mi_lp_comm_get_unique_id(buf) != 0:
                raise RuntimeError("mi_lp_comm_get_unique_id: " +
                                   (L.mi_lp_comm_last_error(None) or b"").decode())
            uid = bytes(buf)
            if dist is not None and world > 1:
                box = [uid]
                dist.broadcast_object_list(box, src=0)
                uid = box[0]
        self._buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        self._h = ctypes.c_void_p()
        rc = L.mi_lp_comm_create(self._buf, world, rank, device, ctypes.byref(self._h))
        if rc != 0:
            raise RuntimeError(f"mi_lp_comm_create failed ({rc}): " +
                               (L.mi_lp_comm_last_error(None) or b"").decode())

    @staticmethod
    def unique_id():
        import ctypes
        from . import engine
        buf = (ctypes.c_uint8 * 128)()
        if engine.lib().mi_lp_comm_get_unique_id(buf) != 0:
            raise RuntimeError("mi_lp_comm_get_unique_id failed")
        return bytes(buf)

    def rank(self):
        return self._L.mi_lp_comm_rank(self._h)

    def size(self):
        return self._L.mi_lp_comm_size(self._h)

    def share_bound(self, value, op=MIN):
        import ctypes
        v = ctypes.c_double(value)
        rc = self._L.mi_lp_share_bound(self._h, ctypes.byref(v), op)
        if rc != 0:
            raise RuntimeError(f"mi_lp_share_bound failed ({rc}): " +
                               self._L.mi_lp_comm_last_error(self._h).decode())
        return v.value

    def close(self):
        if self._h:
            self._L.mi_lp_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def max_over_ranks(x, dist=None, device=None):
    """Wall time of the slowest rank (the bench contract's MAX over ranks)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, dist=None, device=None):
    """Total of a per-rank count (iterations or LPs done by every rank)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


# --- single LP split across GPUs -----------------
# One LP over `world` processes: every process loads the same LP and runs the
# same host control flow; process r keeps column block r of [A | I] on its
# GPU (DeviceLp::SetExchange, engine/device_shards.hip). Each per-column
# device operation's results are joined in block order by an all-gather of
# byte strings: the update row's list, the pricing reduced costs, the dual
# ratio test's filtered breakpoints (each block filtered under its own
# bound: the all-reduce(min) of the reference's exchange is implicit in the
# superset), the entering column's coefficient. The engine calls
# allgather_bytes through mi_lp_set_exchange.

def column_blocks(col_starts, world):
    """Column blocks of [A | I] per rank, as DeviceLp::ShardedUpload cuts
    them: balanced by entries, every boundary on a 64-column multiple (so a
    block's mask bits are whole words). Returns world + 1 boundaries."""
    n = len(col_starts) - 1
    total = int(col_starts[n] - col_starts[0])
    bounds = [n] * (world + 1)
    bounds[0] = 0
    s = 1
    for c in range(n):
        if s >= world:
            break
        seen = int(col_starts[c + 1] - col_starts[0])
        if seen * world >= total * s and (c + 1) % 64 == 0:
            bounds[s] = c + 1
            s += 1
    return bounds


def owner_of(col, bounds):
    """Rank whose column block holds `col`."""
    import bisect
    return bisect.bisect_right(bounds, col) - 1


def allgather_bytes(data, sizes, dist, group=None):
    """Every rank's `data` (sizes[r] bytes from rank r, known to all ranks),
    concatenated in rank order: one all-gather of uint8 tensors padded to the
    longest message. On a gloo group the tensors stay on the CPU."""
    import torch
    world = len(sizes)
    cap = max(1, max(sizes))
    buf = torch.zeros(cap, dtype=torch.uint8)
    if data:
        buf[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    outs = [torch.empty(cap, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return b"".join(bytes(outs[r][:sizes[r]].numpy().tobytes()) for r in range(world))


def shm_name(dist, group=None):
    """A fresh shared-memory name chosen by rank 0 and broadcast to the group
    (the only use of the process group on the split's path: setup)."""
    import uuid
    obj = [f"/mi_lp_{uuid.uuid4().hex}" if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def attach_column_split(handle, dist, group=None, transport="shm"):
    """Makes `handle` (engine.LpHandle) this rank's block of one LP split over
    the group (call before handle.load). transport "shm": the joins go through
    the engine's C++ same-node exchange (engine.ShmExchange; the group only
    distributes its name); "gloo": through allgather_bytes on `group` (a
    gloo group: the joined messages are host bytes the engine consumes).
    Returns (rank, world, exchange or None); keep the exchange open while the
    handle solves."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if transport == "shm":
        from . import engine
        x = engine.ShmExchange(shm_name(dist, group), rank, world)
        handle.set_exchange_native(rank, world, x)
        return rank, world, x
    handle.set_exchange(rank, world,
                        lambda data, sizes: allgather_bytes(data, sizes, dist, group))
    return rank, world, None
