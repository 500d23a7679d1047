"""Data-parallel sharding of independent MPC instances over ranks.

Instances within an MPC step are independent (initial conditions, references, perturbed
models), so the batch is split contiguously over the ranks - instance i goes to rank
floor(i * world / total) - and each rank solves its shard with no communication.  The only
collective is one all-gather of the per-instance results after the solve (RCCL over xGMI on
the GPU box with backend "nccl"; gloo in the CPU tests).  The reference has no counterpart: it
solves one instance per MATLAB process (ocpLMPC.m:11-40).
"""
import torch
import torch.distributed as dist


def shard(total, rank, world):
    """[start, stop) of rank's contiguous slice of `total` instances."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError('bad rank/world %d/%d' % (rank, world))
    return total * rank // world, total * (rank + 1) // world


def owner(i, total, world):
    """Rank that owns instance i (inverse of shard)."""
    return ((i + 1) * world - 1) // total


def gather_rows(t, total, world):
    """All-gather the per-rank row blocks of `t` (shape (rows_of_this_rank, ...)) into the full
    (total, ...) tensor on every rank.  Shards may differ by one row: each block is padded to
    ceil(total / world) rows so one fixed-size all_gather suffices."""
    if world == 1:
        return t
    cap = -(-total // world)
    pad = torch.zeros((cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    out = []
    for r in range(world):
        a, b = shard(total, r, world)
        out.append(parts[r][:b - a])
    return torch.cat(out, 0)


def max_over_ranks(x, device, world):
    """max of a host float over ranks (the bench's wall time of the slowest rank)."""
    if world == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
