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
# The engine's column shards (DeviceLp MILP_SHARDS, engine/device_shards.hip)
# join inside one process; across processes the same joins are these
# collectives, one exchange step per dual iteration:
#   * all-reduce(min) of the ratio test's Harris bound over the shards,
#   * an all-gather of each shard's candidate breakpoints (few), concatenated
#     in rank (= column block) order, the order the host replays them in,
#   * a broadcast of the entering column a_q from the rank that owns it.

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


def min_bound(bound, dist=None, device=None):
    """All-reduce(min) of the per-shard Harris bound (the filter key)."""
    return share_bound(bound, dist, device)


def gather_candidates(cols, coeffs, dist=None, device=None):
    """All-gather of the per-rank candidate lists (global column ids and
    their update-row coefficients), concatenated in rank order. Lists are
    padded to the longest one for the fixed-size collective."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return list(cols), list(coeffs)
    world = dist.get_world_size()
    n = torch.tensor([len(cols)], dtype=torch.int64, device=device or "cpu")
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    cap = max(int(s.item()) for s in sizes)
    c = torch.full((max(cap, 1),), -1, dtype=torch.int64, device=device or "cpu")
    v = torch.zeros((max(cap, 1),), dtype=torch.float64, device=device or "cpu")
    if cols:
        c[:len(cols)] = torch.tensor(list(cols), dtype=torch.int64)
        v[:len(coeffs)] = torch.tensor(list(coeffs), dtype=torch.float64)
    cs = [torch.empty_like(c) for _ in range(world)]
    vs = [torch.empty_like(v) for _ in range(world)]
    dist.all_gather(cs, c)
    dist.all_gather(vs, v)
    out_c, out_v = [], []
    for r in range(world):
        k = int(sizes[r].item())
        out_c += [int(x) for x in cs[r][:k].tolist()]
        out_v += [float(x) for x in vs[r][:k].tolist()]
    return out_c, out_v


def broadcast_column(values, owner, dist=None, device=None):
    """The entering column a_q (dense, m values) from the rank that owns it."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return list(values)
    t = torch.tensor(list(values), dtype=torch.float64, device=device or "cpu")
    dist.broadcast(t, src=owner)
    return [float(x) for x in t.tolist()]
