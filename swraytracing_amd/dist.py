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


def shard_bounds(n_total: int, weights) -> list[tuple[int, int]]:
    """Contiguous blocks [lo, hi) of n_total packets in proportion to
    `weights` (one per rank, >= 0): rank r's block ends at
    round(n_total * sum(weights[:r+1]) / sum(weights)).  The same float
    operations on every rank, so every rank computes the same partition."""
    w = [float(v) for v in weights]
    if not w or any(v < 0 for v in w) or sum(w) <= 0:
        raise ValueError("weights must be >= 0 with a positive sum")
    tot = sum(w)
    ends, acc = [], 0.0
    for v in w:
        acc += v
        ends.append(int(round(n_total * acc / tot)))
    ends[-1] = n_total
    out, lo = [], 0
    for e in ends:
        hi = max(lo, min(e, n_total))
        out.append((lo, hi))
        lo = hi
    return out


def owner_bounds(n_total: int, world: int, owner_weight: float) -> list[tuple[int, int]]:
    """The PDE-owner partition: rank 0 steps the PDE and takes `owner_weight`
    packets for every 1 a receiving rank takes (OwnerLink)."""
    if world == 1:
        return [(0, n_total)]
    return shard_bounds(n_total, [owner_weight] + [1.0] * (world - 1))


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


def gather_packets(ctx, n_total: int, world: int, rank: int, group=None, bounds=None):
    """Gather every rank's device-resident packets into the full (n_total, 2)
    x and k on rank 0, in global packet order (shard_range layout), without a
    host round trip on the sending side: libswrt writes the shard's state in
    original order straight into a torch device buffer (swrt_packets_get_device,
    on the library's packet stream), and one all_gather of the (4, ceil(n/world))
    blocks runs with that stream as torch's current stream, so the collective
    (RCCL on "nccl"; gloo stages through the host) is ordered after the write
    with no synchronisation.  Returns (x, k) numpy arrays on rank 0, None
    elsewhere.  ``bounds``: each rank's [lo, hi) (shard_bounds; default the
    even shard_range blocks)."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device())
    bounds = bounds or [shard_range(n_total, world, r) for r in range(world)]
    maxn = max(1, max(hi - lo for lo, hi in bounds))
    lo, hi = bounds[rank]
    if ctx.packets_count() != hi - lo:
        raise ValueError(f"rank {rank} holds {ctx.packets_count()} packets, its shard is {hi - lo}")
    stream = torch.cuda.ExternalStream(ctx.stream(), device=dev)
    with torch.cuda.stream(stream):
        buf = torch.zeros((4, maxn), dtype=torch.float64, device=dev)  # rows x, y, k, l
        if hi > lo:
            ctx.packets_get_device(buf.data_ptr(), buf.data_ptr() + 2 * maxn * 8, maxn)
        out = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(out, buf, group=group)
        if rank != 0:
            torch.cuda.current_stream().synchronize()
            return None
        full = torch.cat([out[r][:, : bounds[r][1] - bounds[r][0]] for r in range(world)], dim=1).cpu().numpy()
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


def _host_wait(work):
    """Block the host until an asynchronous collective has completed, without
    queueing a device-side wait on any stream (Work.wait() on "nccl" would make
    the current stream wait on RCCL's); then surface its error, if any."""
    import time
    while not work.is_completed():
        time.sleep(0)
    with _default_stream():
        work.wait()


def _default_stream():
    import contextlib

    import torch
    if not torch.cuda.is_available():
        return contextlib.nullcontext()
    return torch.cuda.stream(torch.cuda.default_stream())


class OwnerLink:
    """The PDE-owner driver's per-step hand-off (qg2layersw_raytrace.m:152-197
    sharded with the PDE on ONE rank): the packets read only the top layer of
    qk (:186-188), so the owner rank sends that layer's spectral PV (the
    (2kmax+1)(kmax+1) half plane, 2.1 MB at 512^2) and the step's dt after
    every PDE step, and every other rank builds its snapshots from it
    (swrt_snapshot_qk: bit for bit the owner's swrt_qg_snapshot) instead of
    stepping the replicated 2-layer PDE.

    "nccl" (RCCL over xGMI): the half plane goes by one broadcast of a device
    buffer per step, with dt appended to it; dt also goes by a host-side
    broadcast on a gloo group, because a receiving host needs it to queue its
    packets and reading it back from the device would wait behind the packet
    launches that hold the GPU.  "gloo": one host buffer carries both.
    ``nbuf`` buffers in turn (the latest qk, the previous one, and the ones a
    receiver has not read yet).  No stream of the library ever waits on a
    torch or RCCL stream: the owner's export into a buffer is fenced on the
    host against the broadcast that last read it, the owner's broadcast is
    asynchronous (its completion polled on the host, never waited for on the
    packet stream), and a receiver's snapshot reads a buffer only after the
    host has seen its broadcast complete (ReceiverLoop).  A cross-stream wait
    on ROCm costs 0.1-0.2 ms per step while packet launches hold the GPU
    (tools/owner_legs.py)."""

    def __init__(self, nx, backend, owner=0, group=None, device=None, nbuf=5):
        """``device``: device buffers (default: with "nccl"); True with
        "gloo" runs the device form over gloo's CUDA-tensor broadcast (the
        tests' way to exercise it with ranks sharing one GPU).  ``nbuf``:
        buffers in turn (>= 2: the latest qk and the previous one; a receiver's
        fenced snapshots need ReceiverLoop.ahead + mark_every of them)."""
        import torch
        kmax = nx // 2 - 1
        self.nx = int(nx)
        self.nh = (2 * kmax + 1) * (kmax + 1)
        self.owner, self.group = owner, group
        self.device = (backend == "nccl") if device is None else bool(device)
        dev = torch.device("cuda", torch.cuda.current_device()) if self.device else torch.device("cpu")
        self.stream = torch.cuda.Stream(device=dev) if self.device else None
        # [qk half plane (2*nh doubles) | dt]
        self.nbuf = max(2, int(nbuf))
        self.bufs = [torch.zeros(2 * self.nh + 1, dtype=torch.float64, device=dev) for _ in range(self.nbuf)]
        self.cur = 0  # the buffer holding the latest qk
        self.dt_group = None
        self._dt = [torch.zeros(1, dtype=torch.float64) for _ in range(2)]
        self._sent = [None] * self.nbuf if self.device else None
        self._dt_work = None
        if self.device:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                self.dt_group = dist.new_group(backend="gloo")  # (a collective: every rank builds the link)

    def _on_stream(self):
        import contextlib

        import torch
        return torch.cuda.stream(self.stream) if self.device else contextlib.nullcontext()

    def _export(self, ctx, b, dt=0.0):
        if self.device:
            # host-fenced: the broadcast that last read this buffer (nbuf
            # publishes ago) is waited for here, so the QG stream never waits
            # on the link stream (see swrt_qg_export dst_mode 2)
            i = next(k for k, x in enumerate(self.bufs) if x is b)
            if self._sent is not None and self._sent[i] is not None:
                _host_wait(self._sent[i])
                self._sent[i] = None
            ctx.qg_export(b.data_ptr(), which=0, layer=0, stream=self.stream.cuda_stream, tail=dt, fenced=True)
        else:
            ctx.qg_export(b.numpy(), which=0, layer=0, tail=dt)

    def _bcast(self, b, async_op=False):
        import torch.distributed as dist
        with self._on_stream():
            return dist.broadcast(b, src=self.owner, group=self.group, async_op=async_op)

    def _send_dt(self, dt):
        if not self.device:
            return  # (the host buffer carried it)
        import torch.distributed as dist
        if self._dt_work is not None:
            self._dt_work.wait()
        t = self._dt[self.cur & 1]
        t[0] = float(dt)
        self._dt_work = dist.broadcast(t, src=self.owner, group=self.dt_group, async_op=True)

    def _recv_dt(self, b):
        if not self.device:
            return float(b[-1])
        import torch.distributed as dist
        t = self._dt[self.cur & 1]
        dist.broadcast(t, src=self.owner, group=self.dt_group)
        return float(t[0])

    def bind_owner(self, ctx):
        """The owner's link runs on the context's packet stream (device form):
        the export is ordered after the QG stream by the library's own events,
        the broadcast follows it in stream order, and no stream of the
        library ever waits on a torch stream's event (tools/owner_legs.py
        --owner-export: a link stream of its own made the owner's step 1.1-2x
        slower and erratic while packet launches held the GPU).  A PDE owner
        without packets has nothing else on that stream."""
        if self.device:
            import torch
            self.stream = torch.cuda.ExternalStream(ctx.stream())
        return self

    def _next(self):
        return (self.cur + 1) % self.nbuf

    def seed(self, ctx):
        """Every rank: the model's initial qk as the 'previous' buffer (all
        ranks hold the same initial state)."""
        self._export(ctx, self.bufs[self.cur])

    def publish(self, ctx, dt):
        """Owner: the committed current qk's top layer and dt to every rank."""
        i = self._next()
        b = self.bufs[i]
        self._export(ctx, b, dt)
        # asynchronous: RCCL's stream waits for the export queued so far on
        # self.stream, and nothing waits for RCCL's stream on the device; the
        # buffer's next export polls the work on the host (_export)
        work = self._bcast(b, async_op=self._sent is not None)
        if self._sent is not None:
            self._sent[i] = work
        self.cur = i
        self._send_dt(dt)

    def receive(self, wait=False):
        """Receiver: the owner's next (qk, dt); returns dt (a host float).
        The qk half plane may still be in flight (device) — the snapshot that
        reads it waits for it on the device — unless ``wait``: then the host
        waits for it here (see snapshot's ``fenced``)."""
        b = self.bufs[self._next()]
        self._bcast(b)
        self.cur = self._next()
        dt = self._recv_dt(b)
        if wait and self.device:
            self.stream.synchronize()
        return dt

    def close(self):
        if self._dt_work is not None:
            self._dt_work.wait()
            self._dt_work = None
        for i, w in enumerate(self._sent or []):
            if w is not None:
                _host_wait(w)
                self._sent[i] = None

    def snapshot(self, ctx, slot, which, L, K_d2, shear, k_scale, ny_period, fenced=False):
        """grid_U of the latest (which 0) or the previous (1) qk into `slot`.
        ``fenced``: the caller guarantees the order itself — the buffer's
        broadcast has completed (receive(wait=True)) and its next fill comes
        only after this snapshot has run (ReceiverLoop's pacing) — so no event
        ties the library's stream to the link's.  (A cross-stream wait on the
        link stream measured ~0.2 ms per step on ROCm beside packet launches:
        every hop of a barrier between queues waits on the command processor,
        tools/owner_legs.py.)"""
        b = self.bufs[self.cur if which == 0 else (self.cur - 1) % self.nbuf]
        if self.device:
            ctx.snapshot_qk(slot, b.data_ptr(), self.nx, L, K_d2, shear, k_scale, ny_period,
                            stream=None if fenced else self.stream.cuda_stream)
        else:
            ctx.snapshot_qk(slot, b[: 2 * self.nh].numpy(), self.nx, L, K_d2, shear, k_scale, ny_period)
