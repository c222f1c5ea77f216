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


def device_index(local: int) -> int:
    """GPU of a local rank: one rank per GPU.  With fewer GPUs than ranks
    (a gloo rehearsal of N ranks on a one-GPU box) ranks share devices
    round-robin; RCCL itself refuses two ranks on one device."""
    import torch
    n = torch.cuda.device_count()
    return local % n if n else 0


def init(backend: str = "nccl"):
    """Join the process group.  ``backend`` "nccl" is RCCL over xGMI; "gloo"
    runs the same collectives on the host (CPU tests, and rehearsing N ranks
    on fewer GPUs).  VPP_DIST_BACKEND overrides it."""
    import torch
    import torch.distributed as dist
    backend = os.environ.get("VPP_DIST_BACKEND", backend)
    rank, size, local = world()
    # A process started by torch.distributed.run (WORLD_SIZE in the env)
    # joins a group even at world size 1, so the RCCL path runs there too;
    # a plain single process has no group and no collective.
    if "WORLD_SIZE" not in os.environ or dist.is_initialized():
        return
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)


def backend() -> str:
    import torch.distributed as dist
    return dist.get_backend() if dist.is_initialized() else "none"


def shard(rank: int, n_per_rank: int) -> tuple:
    """First stream index and count of this rank's packets."""
    return rank * n_per_rank, n_per_rank


def merge_counters(counters):
    """All-reduce (sum) an int64 counter tensor in place across the ranks of
    the group (any size, 1 included).  With gloo the collective runs on the
    host: device counters go through a host copy (the rehearsal path; RCCL
    reduces them in HBM, on the caller's current stream's order)."""
    import torch.distributed as dist
    if dist.is_initialized():
        if counters.is_cuda and dist.get_backend() == "gloo":
            h = counters.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            counters.copy_(h)
        else:
            dist.all_reduce(counters, op=dist.ReduceOp.SUM)
    return counters


def max_over_ranks(value, device=None):
    """Max of a float (or a list of floats, elementwise) over the ranks."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return value
    if dist.get_backend() == "gloo":
        device = None
    vals = list(value) if isinstance(value, (list, tuple)) else [value]
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out = [float(x) for x in t.cpu()]
    return out if isinstance(value, (list, tuple)) else out[0]
