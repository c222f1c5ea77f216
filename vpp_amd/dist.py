"""Multi-GPU data parallelism over packets.

One process per GPU (torch.distributed, launched by torch.distributed.run).
Packets shard contiguously: rank r owns stream packets [r*N, (r+1)*N) of the
counter-based generator, so no packet data ever crosses GPUs.  The rule table
is replicated (compiled and uploaded by every rank).  The only collective is
the integer-sum all-reduce of the per-rule hit counters (RCCL over xGMI with
the "nccl" backend; gloo on CPU in tests): (R+1) x 8 B, latency-bound, and
bit-exact in any reduction order.
"""
from __future__ import annotations

import os


def world() -> tuple:
    """(rank, world_size, local_rank) from the torch.distributed.run env."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl"):
    import torch
    import torch.distributed as dist
    rank, size, local = world()
    if size <= 1 or dist.is_initialized():
        return
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)


def shard(rank: int, n_per_rank: int) -> tuple:
    """First stream index and count of this rank's packets."""
    return rank * n_per_rank, n_per_rank


def merge_counters(counters):
    """All-reduce (sum) an int64 counter tensor in place across ranks."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM)
    return counters


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
