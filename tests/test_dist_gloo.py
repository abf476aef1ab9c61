"""Multi-process path on CPU: world_size-2 and -4 gloo (no GPU needed).

Covers the sharding / gather / max-reduce logic that bench.py and the
distributed driver use; the per-shard physics is the (bit-exact) oracle so
the gathered result must equal a single-process run exactly."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from swraytracing_amd.dist import shard_range


def test_shard_range_partitions_exactly():
    for n in (0, 1, 7, 10, 1_000_003):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = shard_range(n, world, r)
                assert 0 <= lo <= hi <= n
                assert hi - lo in (n // world, n // world + 1)
                seen.append((lo, hi))
            assert seen[0][0] == 0 and seen[-1][1] == n
            assert all(seen[i][1] == seen[i + 1][0] for i in range(world - 1))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import torch.distributed as dist

    from oracle import swrt_oracle as orc
    from swraytracing_amd.dist import gather_to_root, max_over_ranks, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(146)
        nx, L = 32, 2 * np.pi
        X = np.arange(nx) * L / nx
        XX, YY = np.meshgrid(X, X, indexing="ij")
        psi = 0.05 * np.cos(2 * XX + YY) + 0.03 * np.sin(XX - 3 * YY)
        fields = orc.spectral_scheme_fields(L, nx, psi)
        fields.pop("psi")
        x, k = orc.initial_packets(n, L, 4.0, 3.0, 1.0, rng)  # identical on every rank
        lo, hi = shard_range(n, world, rank)
        xs, ks, _, _ = orc.leapfrog(x[lo:hi], k[lo:hi], 0.01, 5, 3.0, 1.0, orc.GridField(fields, L / nx))
        full_x = gather_to_root(xs, n, world, rank)
        full_k = gather_to_root(ks, n, world, rank)
        tmax = max_over_ranks(float(rank) + 0.5)
        if rank == 0:
            xr, kr, _, _ = orc.leapfrog(x, k, 0.01, 5, 3.0, 1.0, orc.GridField(fields, L / nx))
            q.put((bool(np.array_equal(full_x, xr) and np.array_equal(full_k, kr)), tmax))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 101), (2, 64), (4, 101)])
def test_gloo_shard_gather_matches_single_process(world, n):
    """world ranks (gloo), ragged shards when world does not divide n."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    ok, tmax = q.get(timeout=10)
    assert ok
    assert tmax == world - 0.5  # max over ranks of rank + 0.5


class _ShardCtx:
    """numpy stand-in for the device ode23 stages (swrt_ode23_*) on one shard,
    with the oracle's odefun — so the sharded controller can run on CPU."""

    def __init__(self, y, rhs):
        self.y = y.copy()
        self.rhs = rhs
        self.n = y.size // 4

    def ode23_f1(self, t, tmax, f, Cg, nslots, thr, bump):
        self.F1 = self.rhs(t, self.y)
        return float(np.max(np.abs(self.F1) / np.maximum(np.abs(self.y), thr)))

    def ode23_attempt(self, t, h, tnew, tmax, f, Cg, nslots, thr, bump):
        y = self.y
        F2 = self.rhs(t + h * 0.5, y + self.F1 * (h * 0.5))
        F3 = self.rhs(t + h * 0.75, y + F2 * (h * 0.75))
        h4 = tnew - t
        self.ynew = y + (((self.F1 * (h4 * (2.0 / 9.0))) + F2 * (h4 * (1.0 / 3.0))) + F3 * (h4 * (4.0 / 9.0)))
        self.F4 = self.rhs(tnew, self.ynew)
        fE = ((self.F1 * (-5.0 / 72.0) + F2 * (1.0 / 12.0)) + F3 * (1.0 / 9.0)) + self.F4 * (-1.0 / 8.0)
        return float(np.max(np.abs(fE) / np.maximum(np.maximum(np.abs(y), np.abs(self.ynew)), thr)))

    def ode23_accept(self):
        self.y, self.F1 = self.ynew, self.F4


def _ode23_worker(rank, world, port, n, q):
    import torch.distributed as dist

    from oracle import swrt_oracle as orc
    from swraytracing_amd.dist import allreduce_max_fn, gather_to_root, shard_range
    from swraytracing_amd.integrate import ode23_packets
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(7)
        nx, L, f, Cg = 32, 2 * np.pi, 3.0, 1.0
        X = np.arange(nx) * L / nx
        XX, YY = np.meshgrid(X, X, indexing="ij")
        f1 = orc.spectral_scheme_fields(L, nx, 0.08 * np.cos(2 * XX + YY))
        f2 = orc.spectral_scheme_fields(L, nx, 0.08 * np.cos(2 * XX + YY + 0.4))
        for d_ in (f1, f2):
            d_.pop("psi")
        x, k = orc.initial_packets(n, L, 4.0, f, Cg, rng)
        lo, hi = shard_range(n, world, rank)
        tmax = 0.6
        rhs = orc.raytracing_rhs(f1, f2, f, Cg, tmax, L / nx)
        ys = np.concatenate([x[lo:hi, 0], x[lo:hi, 1], k[lo:hi, 0], k[lo:hi, 1]])
        c = _ShardCtx(ys, rhs)
        st = {}
        ts = ode23_packets(c, (0.0, tmax), tmax, f, Cg, allreduce_max=allreduce_max_fn("gloo"), stats=st)
        m = hi - lo
        local = np.stack([c.y[:m], c.y[m:2 * m], c.y[2 * m:3 * m], c.y[3 * m:]], axis=1)
        full = gather_to_root(local, n, world, rank)
        if rank == 0:
            y0 = np.concatenate([x[:, 0], x[:, 1], k[:, 0], k[:, 1]])
            to, yo = orc.ode23(rhs, [0.0, tmax], y0)
            want = np.stack([yo[:n], yo[n:2 * n], yo[2 * n:3 * n], yo[3 * n:]], axis=1)
            q.put((bool(np.array_equal(ts, to)), bool(np.array_equal(full, want)), st["steps"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_sharded_ode23_takes_the_global_steps(world):
    """ode23's error norm is global: with the packets split over `world` ranks
    and the per-attempt error max-reduced over them, every rank takes exactly
    the single-process step sequence and the gathered state is bit-identical."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ode23_worker, args=(r, world, port, 90, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    same_ts, same_y, steps = q.get(timeout=10)
    assert same_ts and same_y and steps >= 10


def test_owner_bounds_partition_and_weight():
    from swraytracing_amd.dist import owner_bounds, shard_bounds
    for n in (0, 1, 5001, 1_000_000):
        for world in (1, 2, 4, 8):
            for w0 in (0.0, 0.35, 0.5, 1.0, 2.0):
                b = owner_bounds(n, world, w0)
                assert len(b) == world and b[0][0] == 0 and b[-1][1] == n
                assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
                assert all(lo <= hi for lo, hi in b)
                if world > 1 and n >= 1000:
                    n0 = b[0][1] - b[0][0]
                    assert abs(n0 - n * w0 / (w0 + world - 1)) <= 1
    assert shard_bounds(10, [1, 1]) == [(0, 5), (5, 10)]
    with pytest.raises(ValueError):
        shard_bounds(10, [0, 0])


class _FakeQG:
    """The owner's model context: qg_export hands out this step's qk."""

    def __init__(self, nh):
        self.nh = nh
        self.qk = None

    def qg_export(self, dst, which=0, layer=0, stream=None, tail=0.0):
        assert which == 0 and layer == 0 and dst.size == self.nh * 2 + 1
        dst[:-1] = self.qk
        dst[-1] = tail


class _FakeSnap:
    """A receiving rank's context: snapshot_qk records what it was given."""

    def __init__(self):
        self.got = []

    def snapshot_qk(self, slot, qk, nx, L, K_d2, shear, k_scale, ny_period, stream=None):
        self.got.append((slot, qk.copy(), (nx, L, K_d2, shear, k_scale, ny_period)))


def _owner_link_worker(rank, world, port, q):
    import torch.distributed as dist

    from swraytracing_amd.dist import OwnerLink
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nx = 16
        link = OwnerLink(nx, "gloo")
        rng = np.random.default_rng(11)  # the same stream on every rank: rank 0 sends, the others check
        seq = [rng.standard_normal(2 * link.nh) for _ in range(6)]
        dts = [0.01 * (1 + i) for i in range(5)]
        if rank == 0:
            m = _FakeQG(link.nh)
            m.qk = seq[0]
            link.seed(m)
            for i, dt in enumerate(dts):
                m.qk = seq[i + 1]
                link.publish(m, dt)
            ok = True
        else:
            c = _FakeSnap()
            m = _FakeQG(link.nh)
            m.qk = seq[0]
            link.seed(m)  # every rank holds the initial state
            got_dt = []
            for i in range(len(dts)):
                got_dt.append(link.receive())
                if i == 0:
                    link.snapshot(c, 0, 1, 20.0, 3.0, 0.5, 0.3, 2 * nx)  # grid_U(prev_qk) on the first active step
                link.snapshot(c, 1, 0, 20.0, 3.0, 0.5, 0.3, 2 * nx)
            want = [(0, seq[0])] + [(1, seq[i + 1]) for i in range(len(dts))]
            ok = (got_dt == dts and len(c.got) == len(want)
                  and all(s == ws and np.array_equal(a, wa) for (s, a, _), (ws, wa) in zip(c.got, want))
                  and all(p == (nx, 20.0, 3.0, 0.5, 0.3, 2 * nx) for _, _, p in c.got))
        flags = [None] * world
        dist.all_gather_object(flags, ok)
        if rank == 0:
            q.put(all(flags))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_owner_link_hands_every_step_to_every_rank(world):
    """The PDE-owner hand-off (dist.OwnerLink, gloo): each PDE step's top-layer
    qk and dt, published by rank 0 after the step, reach every other rank in
    order, with the previous step's qk kept for the first active step's
    grid_U(prev_qk) — the inputs of ReceiverLoop's snapshots (the GPU tests
    check the resulting driver files byte for byte)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_link_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10)


def test_host_wait_polls_without_a_device_wait():
    """dist._host_wait (the owner's fence before refilling a link buffer):
    polls Work.is_completed on the host until the broadcast has completed,
    then calls Work.wait once (outside any stream of the library) to surface
    its error — never a device-side wait before completion."""
    from swraytracing_amd.dist import _host_wait

    class Work:
        def __init__(self, polls, fail=False):
            self.polls, self.fail, self.log = polls, fail, []

        def is_completed(self):
            self.log.append("poll")
            self.polls -= 1
            return self.polls < 0

        def wait(self):
            self.log.append("wait")
            if self.fail:
                raise RuntimeError("broadcast failed")

    w = Work(3)
    _host_wait(w)
    assert w.log == ["poll"] * 4 + ["wait"]
    with pytest.raises(RuntimeError, match="broadcast failed"):
        _host_wait(Work(0, fail=True))
