"""Multi-GPU sharding of a Paxos batch.

Instances are independent (Main.hs:41-45 spawns each instance's actors with
no shared state; acceptors only reply to the requestor, Server.hs:58-71), so
a batch shards by contiguous global-instance-id ranges with no data-path
collective.  Every Philox draw is keyed by the GLOBAL instance id, so the
results are identical for any number of ranks.  The only collective is one
all-reduce (RCCL over xGMI on GPUs, gloo on CPU) of the int64 run-totals
vector at the end of a run.
"""
from __future__ import annotations

from typing import Tuple


def shard_range(rank: int, world: int, first: int, n: int) -> Tuple[int, int]:
    """Global instance range [lo, hi) of `rank` for a batch [first, first+n)."""
    if not (0 <= rank < world):
        raise ValueError("rank %d not in world of %d" % (rank, world))
    lo = first + n * rank // world
    hi = first + n * (rank + 1) // world
    return lo, hi


def allreduce_totals(totals, group=None):
    """Sum a length-16 int64 totals tensor over all ranks (in place)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)
    return totals


def run_sharded(run_fn, cfg, first: int, n: int, rank: int, world: int, device="cpu"):
    """Run this rank's shard with `run_fn(cfg, lo, count) -> totals list[16]`
    and return the all-reduced totals (a torch int64 tensor on `device`)."""
    import torch
    lo, hi = shard_range(rank, world, first, n)
    tot = torch.tensor(run_fn(cfg, lo, hi - lo), dtype=torch.int64, device=device)
    return allreduce_totals(tot)
