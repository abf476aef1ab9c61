"""The multi-stream packet protocol made checkable (swrt_hazard.hpp).

swrt_set_packet_streams(S) runs every LDS-tiled leapfrog launch as S part
launches on S streams that stay unjoined across calls; its safety rests on
"parts write disjoint tile ranges between joins".  These tests run the
library's debug happens-before checker over the call sequences that exercise
that protocol, force the worst overlap with a spin kernel on the extra
streams, and reintroduce the known race of round 3 (the launch after a
re-binning's source-gather sort launch overwriting the buffer it gathers
from) to show the checker reports it before the racy launch is queued.

Reference semantics the bits are pinned to: interpolate.m:43-49 (tap order)
and ode_symplectic.m:23-28 (the step loop), through the C oracle.
"""
import argparse

import numpy as np
import pytest

from oracle import swrt_oracle as orc

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


@pytest.fixture()
def debug_ctx():
    """A context of its own: the session context may carry a QG stream from
    an earlier driver test, and while one is initialised every advance call
    joins the extra packet streams at its end (slot_events), which hides the
    cross-call overlap these tests are about."""
    import swraytracing_amd as sw
    import swraytracing_amd._lib as L
    ctx = sw.Context(0)
    yield ctx, L
    ctx.close()


def _bench_workload(ctx, packets):
    import bench
    bench._imports()
    args = argparse.Namespace(nx=512, packets=packets, world=1, rank=0, seed=146, mode="blend")
    return bench, bench.build_workload(ctx, args, 0, packets, packets)


def _run_calls(ctx, bench, w, calls, sub=5):
    ctx.packets_set(w["x"], w["k"])
    for _ in range(calls):
        bench.step(ctx, w, sub)
    return ctx.packets_get()


def test_adversarial_overlap_bitexact_and_checker_silent(debug_ctx, oracle_lib):
    """A ~200 us sleep kernel before every extra-stream part launch: call k's
    extra parts run entirely under call k+1's packet-stream part — and under
    the sort launch that follows each re-binning, which gathers its input from
    any slot.  12 calls of the bench step (5 substeps, re-binning every 20
    steps: 3 re-binnings, each with its sort launch) give the bits of one
    stream and of the C oracle, and the checker (on for the whole run) finds
    every cross-stream access ordered."""
    ctx, L = debug_ctx
    bench, w = _bench_workload(ctx, 300_000)
    ctx.set_locality(20, 0)
    ctx.set_packet_streams(1)
    x1, k1 = _run_calls(ctx, bench, w, 12)
    ctx.set_packet_streams(2)
    ctx.debug_set(L.DEBUG_HAZARD_CHECK, 1)
    ctx.debug_set(L.DEBUG_SPIN_US, 200)
    xs, ks = _run_calls(ctx, bench, w, 12)
    checks = ctx.debug_get(L.DEBUG_HAZARD_CHECKS)
    assert checks > 1000, checks  # the checker saw the part launches
    assert _bits_equal(x1, xs) and _bits_equal(k1, ks)
    p0, p1 = ctx.get_field_grid(0, 512), ctx.get_field_grid(1, 512)
    idx = np.sort(np.random.default_rng(11).choice(300_000, 1200, replace=False))
    xo, ko = w["x"][idx], w["k"][idx]
    for _ in range(12):
        xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.1, 0.2, 512, 1024, w["L"] / 512, orc.BUMP_QG, xo, ko,
                                           w["dt"] / 5, 5, w["f"], w["gH"])
    np.testing.assert_array_equal(xs[idx], xo)
    np.testing.assert_array_equal(ks[idx], ko)


def test_checker_catches_the_pre_third_buffer_race(debug_ctx):
    """The ordering before the third packet buffers (test-only switch): the
    launch after a sort launch writes the buffer that sort launch's extra-
    stream parts gather from.  With the checker on, that launch is refused
    (SWRT_ERR_STATE naming both accesses) before it is queued."""
    import swraytracing_amd as sw
    ctx, L = debug_ctx
    bench, w = _bench_workload(ctx, 300_000)
    ctx.set_locality(20, 0)
    ctx.set_packet_streams(2)
    ctx.debug_set(L.DEBUG_LEGACY_PARK, 1)
    ctx.debug_set(L.DEBUG_HAZARD_CHECK, 1)
    ctx.packets_set(w["x"], w["k"])
    bench.step(ctx, w, 5)  # re-binning + the sort launch (gathers through src_idx)
    with pytest.raises(sw.SwrtError) as ei:
        bench.step(ctx, w, 5)  # its output buffer is the one the sort launch reads
    msg = str(ei.value)
    assert "SWRT_ERR_STATE" in msg and "hazard" in msg and "sort launch" in msg, msg
    ctx.debug_set(L.DEBUG_HAZARD_CHECK, 0)
    ctx.debug_set(L.DEBUG_LEGACY_PARK, 0)
    ctx.synchronize()


def test_the_pre_third_buffer_race_is_real(debug_ctx):
    """The race the checker refuses above changes the result when it is let
    run: with the checker off and a spin kernel before each extra-stream part,
    the legacy ordering corrupts the packets, and the fixed ordering survives
    the same schedule with the one-stream bits.  A demonstration, so it can
    only show the race when the two packet streams really run side by side.
    ROCm multiplexes streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4
    here), and two streams sharing one run in order; twice in round 6 every
    spin missed, in sessions that had created other streams first.  The test
    then skips rather than claim a race it could not show."""
    ctx, L = debug_ctx
    bench, w = _bench_workload(ctx, 300_000)
    ctx.set_locality(20, 0)
    ctx.set_packet_streams(1)
    x1, k1 = _run_calls(ctx, bench, w, 6)
    ctx.set_packet_streams(2)
    ctx.debug_set(L.DEBUG_LEGACY_PARK, 1)
    corrupted = False
    for spin in (200, 2000, 5000, 10000):
        ctx.debug_set(L.DEBUG_SPIN_US, spin)
        xr, kr = _run_calls(ctx, bench, w, 6)
        if not (_bits_equal(x1, xr) and _bits_equal(k1, kr)):
            corrupted = True
            break
    # the fixed ordering under the same schedule: the one-stream bits
    ctx.debug_set(L.DEBUG_LEGACY_PARK, 0)
    xf, kf = _run_calls(ctx, bench, w, 6)
    assert _bits_equal(x1, xf) and _bits_equal(k1, kf)
    if not corrupted:
        pytest.skip("the two packet streams did not overlap under any spin schedule (shared hardware queue?)")


def test_single_launch_after_split_calls_joins_first(debug_ctx):
    """70,000 packets (above the one-stream threshold) advanced by split
    launches, then a call whose launch runs on the packet stream alone — the
    per-packet kernel after swrt_set_locality(0, 0) — then split launches
    again: that launch orders the extra stream's parts of the previous call
    before it (the checker stays silent) and the bits equal one stream's."""
    ctx, L = debug_ctx
    bench, w = _bench_workload(ctx, 70_000)
    out = {}
    for streams in (1, 2):
        ctx.set_packet_streams(streams)
        ctx.set_locality(20, 0)
        ctx.debug_set(L.DEBUG_HAZARD_CHECK, 1 if streams > 1 else 0)
        ctx.debug_set(L.DEBUG_SPIN_US, 100 if streams > 1 else 0)
        ctx.packets_set(w["x"], w["k"])
        for _ in range(3):
            bench.step(ctx, w, 5)
        ctx.set_locality(0, 0)
        bench.step(ctx, w, 5)
        ctx.set_locality(20, 0)
        for _ in range(3):
            bench.step(ctx, w, 5)
        out[streams] = ctx.packets_get()
        ctx.debug_set(L.DEBUG_HAZARD_CHECK, 0)
    assert _bits_equal(out[1][0], out[2][0]) and _bits_equal(out[1][1], out[2][1])


def test_checker_silent_over_the_mixed_call_sequence(debug_ctx):
    """test_packet_streams_bit_identical's call sequence (history frames,
    re-binnings inside and between calls, slot rewrites, multi-interval
    launches, reads, ode23) on 2 streams with the checker on."""
    import swraytracing_amd as sw
    ctx, L = debug_ctx
    bench, w = _bench_workload(ctx, 300_000)
    p0, p1 = ctx.get_field_grid(0).copy(), ctx.get_field_grid(1).copy()
    h = w["dt"] / 5
    for streams in (2,):
        ctx.set_packet_streams(streams)
        ctx.set_locality(20, 0)
        ctx.debug_set(L.DEBUG_HAZARD_CHECK, 1)
        ctx.set_field_grid(0, p0, 512, w["L"], 1024)
        ctx.set_field_grid(1, p1, 512, w["L"], 1024)
        ctx.packets_set(w["x"], w["k"])
        ctx.history_reset()
        for _ in range(7):
            ctx.advance(h, 5, w["f"], w["gH"], nslots=2, alpha0=0.1, dalpha=0.2, bump=orc.BUMP_QG, save_every=5)
        ctx.packets_get()
        ctx.history()
        ctx.set_field_grid(1, p0, 512, w["L"], 1024)
        ctx.set_field_grid(2, p1, 512, w["L"], 1024)
        ctx.advance_intervals([h, 1.1 * h], 5, w["f"], w["gH"], alpha0=0.1, dalpha=0.2, bump=orc.BUMP_QG)
        ctx.advance(h, 3, w["f"], w["gH"], nslots=2, alpha0=0.1, dalpha=0.2, bump=orc.BUMP_QG)
        ctx.packets_get()
        ctx.set_field_grid(1, p1, 512, w["L"], 1024)
        sw.ode23_packets(ctx, (0.0, 5 * h), 5 * h, w["f"], 1.0, stats={})
        ctx.packets_get()
        assert ctx.debug_get(L.DEBUG_HAZARD_CHECKS) > 0
        ctx.debug_set(L.DEBUG_HAZARD_CHECK, 0)


def test_checker_refuses_a_skewed_cycle_end_share(debug_ctx):
    """Round 4's hang (profiles/r04_stream_split): the launch that ends a
    re-binning cycle split its tiles unevenly between the two packet streams
    (SWRT_DEBUG_SHARE_SKEW: 2/3 : 1/3), so its packet-stream part took tiles
    the other stream's part of the previous call could still be writing.  The
    checker enumerates the tiles each part launch takes with the device's own
    mapping (swrt_share.hpp), so it refuses that launch before anything is
    queued; the skew is refused outright without the checker.  Reference
    semantics guarded: ode_symplectic.m:18-21 — packets are independent, so
    any tile schedule must give the same bits, which only a race can break."""
    import swraytracing_amd as sw
    ctx, L = debug_ctx
    bench, w = _bench_workload(ctx, 300_000)
    ctx.set_locality(20, 0)
    ctx.set_packet_streams(2)
    with pytest.raises(sw.SwrtError) as ei:
        ctx.debug_set(L.DEBUG_SHARE_SKEW, 1)  # not without the checker
    assert "SWRT_ERR_STATE" in str(ei.value)
    ctx.debug_set(L.DEBUG_HAZARD_CHECK, 1)
    ctx.debug_set(L.DEBUG_SHARE_SKEW, 1)
    ctx.packets_set(w["x"], w["k"])
    for _ in range(3):  # the cycle's first three launches: the product share
        bench.step(ctx, w, 5)
    with pytest.raises(sw.SwrtError) as ei:
        bench.step(ctx, w, 5)  # the cycle-ending launch, skewed
    msg = str(ei.value)
    assert "SWRT_ERR_STATE" in msg and "hazard" in msg and "skewed" in msg, msg
    # nothing was queued: after a join the state is the one-stream state of 15 steps
    ctx.debug_set(L.DEBUG_SHARE_SKEW, 0)
    ctx.debug_set(L.DEBUG_HAZARD_CHECK, 0)
    xa, ka = ctx.packets_get()
    ctx.set_packet_streams(1)
    x1, k1 = _run_calls(ctx, bench, w, 3)
    assert _bits_equal(x1, xa) and _bits_equal(k1, ka)


@pytest.mark.parametrize("delta", [1000, -7])
def test_corrupted_tile_count_is_an_error_not_a_hang(debug_ctx, delta):
    """One tile count corrupted before a re-binning's scan (on the packet
    stream, with the second stream's parts in flight): the scan's own check
    (counts >= 0 summing to the packets, bin_scan_kernel) leaves an empty
    binning, so no launch walks a bad packet range, and the next host
    synchronisation returns SWRT_ERR_STATE; the packet state stays refused
    until swrt_packets_set, after which the run gives the one-stream bits."""
    import swraytracing_amd as sw
    ctx, L = debug_ctx
    bench, w = _bench_workload(ctx, 300_000)
    ctx.set_locality(20, 0)
    ctx.set_packet_streams(1)
    x1, k1 = _run_calls(ctx, bench, w, 6)
    ctx.set_packet_streams(2)
    ctx.packets_set(w["x"], w["k"])
    for _ in range(2):
        bench.step(ctx, w, 5)
    ctx.debug_set(L.DEBUG_CORRUPT_COUNT, delta)
    for _ in range(6):
        bench.step(ctx, w, 5)  # queued asynchronously: the error surfaces at the next sync
    with pytest.raises(sw.SwrtError) as ei:
        ctx.synchronize()
    assert "SWRT_ERR_STATE" in str(ei.value) and "binning" in str(ei.value)
    with pytest.raises(sw.SwrtError):
        ctx.packets_get()
    x2, k2 = _run_calls(ctx, bench, w, 6)  # packets_set clears it
    assert _bits_equal(x1, x2) and _bits_equal(k1, k2)


def test_corrupted_binning_in_ode23_refuses_the_packets_until_reset(debug_ctx):
    """The same device check inside the drivers' ode23 (its calls re-bin every
    2nd interval): the call that meets it returns SWRT_ERR_STATE, and every
    entry point that reads the packets — the ode23 calls, swrt_packets_get(_device),
    swrt_advance — refuses the lost state until swrt_packets_set, instead of
    integrating it (or unpermuting it through a stale permutation) and
    returning SWRT_OK.  qgsw_raytrace.m:149 semantics are unaffected: after
    packets_set the interval gives the bits of a fresh context."""
    import torch

    import swraytracing_amd as sw
    ctx, L = debug_ctx
    bench, w = _bench_workload(ctx, 300_000)
    f, Cg, dt = w["f"], 1.0, w["dt"]
    run = lambda: ctx.ode23_run(0.0, dt, dt, f, Cg, 2, 1e-3, 1e-6, sw.BUMP_QG)  # noqa: E731
    ctx.packets_set(w["x"], w["k"])
    ts_ref, st_ref = run()
    x_ref, k_ref = ctx.packets_get()
    ctx.packets_set(w["x"], w["k"])
    ctx.debug_set(L.DEBUG_CORRUPT_COUNT, 1000)
    with pytest.raises(sw.SwrtError, match="binning"):
        for _ in range(3):  # the next re-binning meets the corrupted count
            run()
    buf = torch.zeros((4, 300_000), dtype=torch.float64, device="cuda")
    refused = {
        "ode23_run": run,
        "ode23_f1": lambda: ctx.ode23_f1(0.0, dt, f, Cg, 2, 1e-3, sw.BUMP_QG),
        "ode23_attempt": lambda: ctx.ode23_attempt(0.0, dt / 10, dt / 10, dt, f, Cg, 2, 1e-3, sw.BUMP_QG),
        "ode23_accept": ctx.ode23_accept,
        "packets_get": ctx.packets_get,
        "packets_get_device": lambda: ctx.packets_get_device(buf.data_ptr(), buf.data_ptr() + 2 * 300_000 * 8,
                                                             300_000),
        "advance": lambda: bench.step(ctx, w, 5),
    }
    for name, call in refused.items():
        with pytest.raises(sw.SwrtError, match="lost"):
            call()
    torch.cuda.synchronize()
    ctx.packets_set(w["x"], w["k"])
    ts, st = run()
    x, k = ctx.packets_get()
    assert _bits_equal(ts, ts_ref) and st == st_ref
    assert _bits_equal(x, x_ref) and _bits_equal(k, k_ref)
