"""Stripe sharding across ranks (one process per GPU).

Stripes are independent, so a batch is split into contiguous
stripe ranges, one per rank, with no data-path collective.  The process group
carries only the barrier around the timed region and the max-over-ranks
reduction of the elapsed time (RCCL on GPUs, gloo in the CPU tests).
"""
from __future__ import annotations

from typing import Tuple


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, start+count) stripe range of `rank`; sizes differ by
    at most one stripe and the ranges tile [0, total) in rank order."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def max_over_ranks(value: float, device=None) -> float:
    """MAX-allreduce of a float across the default process group (identity
    when torch.distributed is not initialised)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
