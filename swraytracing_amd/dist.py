"""Packet sharding across GPUs (one process per GPU, torch.distributed).

The packet ODEs are independent given the background (ode_symplectic.m:18-21
has no packet-packet coupling), so the ensemble is split into contiguous
shards, the field is replicated (every rank prepares the same snapshots from
the same spectral coefficients, or rank 0 broadcasts them), and the only
collective is the gather of trajectories to rank 0 for the packet_x/k.bin
writer.  Backend "nccl" is RCCL on ROCm (xGMI); "gloo" runs the
same code on CPU tensors for tests.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of rank `rank` (sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    q, r = divmod(n_total, world)
    lo = rank * q + min(rank, r)
    hi = lo + q + (1 if rank < r else 0)
    return lo, hi


def _device_for(backend: str):
    import torch
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_to_root(local: np.ndarray, n_total: int, world: int, rank: int, backend: str = "gloo",
                   group=None):
    """Gather each rank's (n_local, ...) fp64 shard into the full (n_total, ...)
    array on rank 0, in global packet order (shard_range layout).  Returns the
    array on rank 0 and None elsewhere.  One all_gather of equal-size padded
    blocks (RCCL on "nccl")."""
    import torch
    import torch.distributed as dist
    local = np.ascontiguousarray(local, dtype=np.float64)
    tail = local.shape[1:]
    width = int(np.prod(tail)) if tail else 1
    maxn = -(-n_total // world)
    dev = _device_for(backend)
    buf = torch.zeros((maxn, width), dtype=torch.float64, device=dev)
    buf[: local.shape[0]] = torch.from_numpy(local.reshape(local.shape[0], width)).to(dev)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    if rank != 0:
        return None
    parts = []
    for r in range(world):
        lo, hi = shard_range(n_total, world, r)
        parts.append(out[r][: hi - lo].cpu().numpy())
    return np.concatenate(parts, axis=0).reshape((n_total,) + tail)


def max_over_ranks(value: float, backend: str = "gloo", group=None) -> float:
    """MAX of a scalar over ranks (bench timing: slowest rank defines the job)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=_device_for(backend))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def allreduce_max_fn(backend: str = "nccl", group=None):
    """A callable v -> MAX over ranks of v, for ode23_packets' global error
    norm when packets are sharded (one 8-byte all_reduce per attempted step,
    RCCL on "nccl")."""
    return lambda v: max_over_ranks(v, backend=backend, group=group)
