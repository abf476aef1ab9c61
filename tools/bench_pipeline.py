"""End-to-end driver throughput: the qg2layersw_raytrace loop at production
size (512^2 x 2 layers, 1e6 packets) with the PDE, the grid_U snapshots and
the packets all on the GPU.  Prints one JSON line with the per-PDE-step time
and its parts (each part timed alone, synchronised):
  pde_ms       swrt_qg_step (update: 8 inverse + 1 paired forward 2-D FFT, AB3)
  cfl_ms       swrt_qg_max_speed (2 inverse 2-D FFTs + max + 8-byte readback)
  snapshot_ms  swrt_qg_snapshot of the current qk (3 inverse 2-D FFTs + pack)
  packets_ms   nsub fused leapfrog substeps of all packets
  step_ms      the whole driver step (cfl, pde, swap + snapshot, packets)
Not the driver's bench (bench.py is)."""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import swraytracing_amd as sw  # noqa: E402
from swraytracing_amd.qg import _packets, initial_q  # noqa: E402


def timed(ctx, fn, reps):
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=512)
    ap.add_argument("--packets", type=int, default=1_000_000)
    ap.add_argument("--nsub", type=int, default=5, help="leapfrog substeps per PDE interval (5: 0.05*dx/U0 each)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ode23", action="store_true", help="also time the drivers' ode23 over one PDE interval")
    ap.add_argument("--ode23-controller", default=None, choices=["library", "python"],
                    help="ode23 step-size controller: in the C library (default) or the Python loop (A/B)")
    ap.add_argument("--one-stream", action="store_true", help="QG PDE on the packet stream (A/B)")
    ap.add_argument("--no-fused", action="store_true", help="separate transforms per QG call (A/B)")
    ap.add_argument("--intervals", type=int, default=1, help="PDE steps whose packet intervals go in one call")
    ap.add_argument("--fixed-dt", action="store_true",
                    help="no CFL rule / U0 read-back per step (the 1-layer driver's loop, qgsw_raytrace.m)")
    args = ap.parse_args()
    nx, L, f, Cg = args.nx, 20.0, 3.0, 1.0
    ctx = sw.Context(0)
    ctx.qg_set_stream(not args.one_stream)
    ctx.qg_set_fused(not args.no_fused)
    rng = np.random.default_rng(5)
    q1 = initial_q(nx, L, 0.2, f / Cg, 10, 30, rng, ndgrid=True)
    qk = np.stack([ctx.g2k(q1), ctx.g2k(-q1)], axis=2)
    model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
    x, k = _packets(args.packets, L, 4.0, f, Cg, rng)
    ens = sw.PacketEnsemble(x, k, L, f, Cg, nx, f / Cg, shear=0.5, k_scale=2 * math.pi / L, nlayers=2, ctx=ctx)
    U0 = model.max_speed()
    dt = 0.25 * (L / nx) / U0
    for _ in range(4):  # past the AB1/AB2 start-up; captures both replay graphs
        model.step(dt)
    model.snapshot(0, which=1, ny_period=2 * nx)
    model.snapshot(1, which=0, ny_period=2 * nx)
    ens.advance(dt, args.nsub)  # warm-up of every kernel

    r = args.steps
    pde = timed(ctx, lambda: model.step(dt), r)
    cfl = timed(ctx, lambda: model.max_speed(), r)
    snap = timed(ctx, lambda: model.snapshot(1, which=0, ny_period=2 * nx), r)
    pk = timed(ctx, lambda: ens.advance(dt, args.nsub), r)

    state = {"dt": dt, "U0": model.max_speed()}

    # the driver's packet branch (qg.py): packet intervals grouped --intervals
    # per call, the PDE running ahead; slot 0 = the current qk's snapshot
    group = sw.qg._IntervalGroup(ctx, ens, args.intervals, args.nsub)
    ctx.swap_slots(0, 1)

    def full_step():
        # the driver's order: CFL rule on the current U0, PDE step, async U0 of
        # the new qk, snapshot + packets queued, then collect U0
        if args.fixed_dt:
            d = state["dt"]
            model.step(d)
            model.snapshot(group.next_slot(), which=0, ny_period=2 * nx)
            group.add(d)
            return
        d, _ = model.cfl_rule(state["dt"], state["U0"], 0.25)
        state["dt"] = d
        model.step(d)
        model.max_speed_async()
        model.snapshot(group.next_slot(), which=0, ny_period=2 * nx)
        group.add(d)
        state["U0"] = model.max_speed_result()

    full = timed(ctx, full_step, r)
    group.flush()
    ode = None
    if args.ode23:
        # one warm-up interval (first-use allocations), then the mean of 5
        ens.advance_ode23(state["dt"], controller=args.ode23_controller)
        st = {}
        reps = 5
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ens.advance_ode23(state["dt"], stats=st, controller=args.ode23_controller)
        ctx.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        ode = {"interval_ms": ms, **st, "rhs_evals": 1 + 3 * st["attempts"],
               "ms_per_rhs_eval": ms / (1 + 3 * st["attempts"])}
    xg, kg = ens.state()
    out = {
        "metric": "driver step time, qg2layersw_raytrace loop on device (PDE + snapshots + packets)",
        "config": {"nx": nx, "layers": 2, "packets": args.packets, "nsub": args.nsub, "steps": r,
                   "qg_stream": not args.one_stream,
                   "qg_fused": not args.no_fused,
                   "packet_intervals": args.intervals, "fixed_dt": args.fixed_dt},
        "pde_ms": pde, "cfl_ms": cfl, "snapshot_ms": snap, "packets_ms": pk, "step_ms": full,
        "packet_steps_per_s": args.packets * args.nsub / (full / 1e3),
        "ode23": ode,
        "finite": bool(np.isfinite(xg).all() and np.isfinite(kg).all()),
    }
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
