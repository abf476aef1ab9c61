"""swrt_advance_intervals (several PDE intervals per launch, interval i
blending slots i and i+1) against the same intervals as separate
swrt_advance calls with the snapshot pair moved to slots (0, 1), and against
the C oracle on a subset.  Bit-exact: the same per-packet arithmetic; only
the launch structure (window re-staging between intervals, one tail and one
in-tile sort per launch) differs."""
import numpy as np
import pytest

import bench
import swraytracing_amd as sw
from oracle import swrt_oracle as orc

pytestmark = pytest.mark.gpu

NX, L, F, GH = 128, 20.0, 3.0, 1.0
KS = 2 * np.pi / L


def _snapshots(n):
    rng = np.random.default_rng(21)
    q = bench.ring_spectrum(NX, 4, 12, rng) * 2e-3
    out = [q]
    for _ in range(n - 1):
        out.append(out[-1] * np.exp(1j * rng.normal(0, 0.1, q.shape)))
    return out


def _set(ctx, slot, qk):
    ctx.set_field_qk(slot, qk, NX, L, F, 0.5, KS, 2 * NX)


def _packets(n, seed=5):
    rng = np.random.default_rng(seed)
    x = L * rng.random((n, 2)) - L / 2
    th = 2 * np.pi * rng.random(n)
    k = 3 * np.sqrt(15.0) * np.stack([np.cos(th), np.sin(th)], axis=1)
    return x, k


def _run_sequential(ctx, snaps, x, k, hs, nsub, save_every):
    ctx.packets_set(x, k)
    ctx.history_reset()
    for i, h in enumerate(hs):
        _set(ctx, 0, snaps[i])
        _set(ctx, 1, snaps[i + 1])
        ctx.advance(h, nsub, F, GH, nslots=2, alpha0=0.5 / nsub, dalpha=1.0 / nsub, bump=sw.BUMP_QG,
                    save_every=save_every)
    xs, ks = ctx.packets_get()
    hx, hk = ctx.history() if save_every else (None, None)
    return xs, ks, hx, hk


def _run_intervals(ctx, snaps, x, k, hs, nsub, save_every):
    ctx.packets_set(x, k)
    ctx.history_reset()
    for i in range(len(hs) + 1):
        _set(ctx, i, snaps[i])
    ctx.advance_intervals(hs, nsub, F, GH, alpha0=0.5 / nsub, dalpha=1.0 / nsub, bump=sw.BUMP_QG,
                          save_every=save_every)
    xs, ks = ctx.packets_get()
    hx, hk = ctx.history() if save_every else (None, None)
    return xs, ks, hx, hk


@pytest.mark.parametrize("nint", [1, 2, 3, 4])
@pytest.mark.parametrize("rebin,kernel", [(20, 0), (10, 0), (7, 0), (20, 1)])
def test_intervals_match_sequential_calls(ctx, nint, rebin, kernel):
    """rebin 20/10 with nsub 5: whole intervals per launch (one launch of up
    to 4 intervals, or launches cut at every re-binning); rebin 7: intervals
    straddle re-binnings (one interval per call path); kernel 1: per-packet
    kernel.  Interval step sizes differ (the CFL rule changes dt)."""
    snaps = _snapshots(nint + 1)
    x, k = _packets(40_000)
    dx = L / NX
    hs = [0.05 * dx / 0.7 * s for s in (1.0, 0.9, 1.1, 1.0)[:nint]]
    ctx.set_kernel(kernel)
    ctx.set_locality(rebin, 0)
    try:
        a = _run_sequential(ctx, snaps, x, k, hs, 5, 5)
        b = _run_intervals(ctx, snaps, x, k, hs, 5, 5)
    finally:
        ctx.set_kernel(0)
        ctx.set_locality(4, 0)
    for u, v in zip(a, b):
        assert u.shape == v.shape
        assert np.array_equal(u.view(np.uint64), v.view(np.uint64))
    assert a[2].shape[0] == nint  # one frame per interval


@pytest.mark.parametrize("sparse", [1, 2])
def test_intervals_match_oracle_subset(ctx, oracle_lib, sparse):
    """Four intervals in one launch vs the C oracle, interval by interval on
    the device-prepared snapshots (a subset of the packets); the dense and the
    sparse launch shape (the window re-staged between intervals in both)."""
    snaps = _snapshots(5)
    x, k = _packets(60_000, seed=9)
    dx = L / NX
    hs = [0.05 * dx / 0.7 * s for s in (1.0, 0.9, 1.1, 1.0)]
    ctx.set_locality(20, 0)
    ctx.set_sparse_tiles(sparse)
    try:
        xs, ks, _, _ = _run_intervals(ctx, snaps, x, k, hs, 5, 0)
        planes = [ctx.get_field_grid(i, NX) for i in range(5)]
    finally:
        ctx.set_sparse_tiles(0)
        ctx.set_locality(4, 0)
    idx = np.sort(np.random.default_rng(3).choice(x.shape[0], 2000, replace=False))
    xo, ko = x[idx], k[idx]
    for i, h in enumerate(hs):
        xo, ko, _, _ = oracle_lib.leapfrog(planes[i], planes[i + 1], 0.1, 0.2, NX, 2 * NX, dx, orc.BUMP_QG, xo, ko,
                                           h, 5, F, GH)
    np.testing.assert_array_equal(xs[idx], xo)
    np.testing.assert_array_equal(ks[idx], ko)


def test_intervals_argument_errors(ctx):
    snaps = _snapshots(2)
    x, k = _packets(100)
    ctx.packets_set(x, k)
    _set(ctx, 0, snaps[0])
    _set(ctx, 1, snaps[1])
    with pytest.raises(RuntimeError):
        ctx.advance_intervals([0.01] * 5, 5, F, GH)        # more intervals than slots
    with pytest.raises(RuntimeError):
        ctx.advance_intervals([0.01, -1.0], 5, F, GH)      # bad step size
    with pytest.raises(RuntimeError):
        ctx.advance_intervals([0.01], 5, F, GH, save_every=3)  # save_every must divide nsub
