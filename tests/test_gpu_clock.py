"""The shader-clock probe behind bench.py's clock_ghz_observed
(swrt_clock_stamp / swrt_clock_ghz): over a region of real packet work it
reports a clock inside the MI355X's range with per-CU clocks that agree, and
it refuses to report without stamps.  Diagnostic only (no reference
counterpart); it normalises the throughput numbers the parity-tested
kernels produce (ode_symplectic.m:23-28 driven by interpolate.m:43-49)."""
import argparse

import pytest

pytestmark = pytest.mark.gpu


def test_clock_probe_over_packet_work(fresh_ctx):
    import bench
    import swraytracing_amd as sw
    ctx = fresh_ctx
    with pytest.raises(sw.SwrtError):
        ctx.clock_ghz()  # no stamps yet
    bench._imports()
    args = argparse.Namespace(nx=512, packets=300_000, world=1, rank=0, seed=146, mode="blend")
    w = bench.build_workload(ctx, args, 0, args.packets, args.packets)
    ctx.packets_set(w["x"], w["k"])
    bench.step(ctx, w, 5)
    ctx.clock_stamp(0)
    for _ in range(20):
        bench.step(ctx, w, 5)
    ctx.clock_stamp(1)
    ghz, spread = ctx.clock_ghz()
    assert 0.8 < ghz < 2.6, ghz
    assert spread < 0.2, spread
