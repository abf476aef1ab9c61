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


def spatial_shard(x, L: float, nx: int, world: int, rank: int) -> np.ndarray:
    """Global indices (ascending) of the packets rank `rank` advances under
    spatial partitioning: those whose position lies in y-strip `rank` of
    `world` equal strips of the periodic domain, strip = floor(cy*world/nx)
    with cell row cy = floor(mod(y, L)/dx) — so a GPU's packets are as dense
    within its strip as the whole ensemble is in the domain, and its occupied
    tiles lie in every x-row of the tile grid (every XCD band of the tile
    order).  Packets are independent (ode_symplectic.m:18-21), so which rank
    advances which packet changes no result; packets that later drift out of
    their strip stay with their rank (correct, only less dense).  SURVEY §8e:
    "spatial tiles for locality"."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    y = np.asarray(x, dtype=np.float64)[:, 1]
    cy = np.minimum(np.floor(np.mod(y, L) / (L / nx)).astype(np.int64), nx - 1)
    return np.nonzero((cy * world) // nx == rank)[0]


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


def gather_packets(ctx, n_total: int, world: int, rank: int, group=None, indices=None):
    """Gather every rank's device-resident packets into the full (n_total, 2)
    x and k on rank 0, in global packet order, without a host round trip on
    the sending side: libswrt writes the shard's state in original order
    straight into a torch device buffer (swrt_packets_get_device, on the
    library's packet stream), and one all_gather of the (5, maxn) blocks — x,
    y, k, l and each packet's global index — runs with that stream as torch's
    current stream, so the collective (RCCL on "nccl"; gloo stages through the
    host) is ordered after the write with no synchronisation.  `indices`: the
    global indices this rank holds (spatial_shard); None = its shard_range
    block.  Returns (x, k) numpy arrays on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device())
    if indices is None:
        lo, hi = shard_range(n_total, world, rank)
        indices = np.arange(lo, hi)
    indices = np.asarray(indices, dtype=np.int64)
    if ctx.packets_count() != indices.shape[0]:
        raise ValueError(f"rank {rank} holds {ctx.packets_count()} packets, its shard is {indices.shape[0]}")
    cnt = torch.tensor([float(indices.shape[0])], dtype=torch.float64, device=dev)
    dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=group)
    maxn = max(1, int(cnt.item()))
    stream = torch.cuda.ExternalStream(ctx.stream(), device=dev)
    with torch.cuda.stream(stream):
        buf = torch.zeros((5, maxn), dtype=torch.float64, device=dev)  # rows x, y, k, l, global index
        buf[4].fill_(-1.0)
        buf[4, : indices.shape[0]] = torch.from_numpy(indices.astype(np.float64)).to(dev)
        ctx.packets_get_device(buf.data_ptr(), buf.data_ptr() + 2 * maxn * 8, maxn)
        out = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(out, buf, group=group)
        if rank != 0:
            torch.cuda.current_stream().synchronize()
            return None
        allb = torch.cat(out, dim=1).cpu().numpy()
    idx = allb[4]
    keep = idx >= 0
    full = np.empty((4, n_total))
    full[:, idx[keep].astype(np.int64)] = allb[0:4, keep]
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
