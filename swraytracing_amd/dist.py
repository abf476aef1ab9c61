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


def gather_packets(ctx, n_total: int, world: int, rank: int, group=None):
    """Gather every rank's device-resident packets into the full (n_total, 2)
    x and k on rank 0, in global packet order (shard_range layout), without a
    host round trip on the sending side: libswrt writes the shard's state in
    original order straight into a torch device buffer (swrt_packets_get_device,
    on the library's packet stream), and one all_gather of the (4, ceil(n/world))
    blocks runs with that stream as torch's current stream, so the collective
    (RCCL on "nccl"; gloo stages through the host) is ordered after the write
    with no synchronisation.  Returns (x, k) numpy arrays on rank 0, None
    elsewhere."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device())
    maxn = max(1, -(-n_total // world))
    lo, hi = shard_range(n_total, world, rank)
    if ctx.packets_count() != hi - lo:
        raise ValueError(f"rank {rank} holds {ctx.packets_count()} packets, its shard is {hi - lo}")
    stream = torch.cuda.ExternalStream(ctx.stream(), device=dev)
    with torch.cuda.stream(stream):
        buf = torch.zeros((4, maxn), dtype=torch.float64, device=dev)  # rows x, y, k, l
        ctx.packets_get_device(buf.data_ptr(), buf.data_ptr() + 2 * maxn * 8, maxn)
        out = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(out, buf, group=group)
        if rank != 0:
            torch.cuda.current_stream().synchronize()
            return None
        full = torch.cat([out[r][:, : shard_range(n_total, world, r)[1] - shard_range(n_total, world, r)[0]]
                          for r in range(world)], dim=1).cpu().numpy()
    return np.ascontiguousarray(full[0:2].T), np.ascontiguousarray(full[2:4].T)


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
