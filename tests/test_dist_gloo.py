"""Multi-process path on CPU: world_size-2 gloo (no GPU needed).

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


@pytest.mark.parametrize("n", [101, 64])
def test_gloo_world2_shard_gather_matches_single_process(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    ok, tmax = q.get(timeout=10)
    assert ok
    assert tmax == 1.5
