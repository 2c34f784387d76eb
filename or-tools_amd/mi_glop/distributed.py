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
