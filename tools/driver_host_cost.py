"""Host cost of one 2-layer driver step (diagnostic): TwoLayerLoop's own call
sequence, each call timed on the host, at a size where the GPU work is
negligible (64^2, 1000 packets) and at the 8-GPU shard size (512^2 x 2,
1.25e5 packets): when the host's time per step approaches the step time the
driver is host-bound.
With --integrator ode23 the step runs the drivers' ode23 over the interval
(the speculative PDE step queued before it, as TwoLayerLoop does): the
"packets" call then holds the host for the whole interval, and the other
calls are the host time between intervals.
usage: python tools/driver_host_cost.py [--steps 200] [--integrator ode23]"""
import argparse
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (one HIP runtime)
import swraytracing_amd as sw  # noqa: E402
import bench  # noqa: E402


def run(nx, N, steps, speculate=True, integrator="leapfrog"):
    L, f, Cg = 20.0, 3.0, 1.0
    rng = np.random.default_rng(7)
    qk1 = bench.ring_spectrum(nx, 1 if nx < 128 else 10, 3 if nx < 128 else 30, rng)
    ctx = sw.Context(0)
    try:
        model = sw.QGModel.two_layer(np.stack([qk1, -qk1], axis=2), nx, f, Cg, L=L, ctx=ctx)
        x = L * rng.random((N, 2)) - L / 2
        k = rng.normal(0.0, 3.0, (N, 2))
        ens = sw.PacketEnsemble(x, k, L, f, Cg, nx, f / Cg, shear=0.5, k_scale=2 * math.pi / L, nlayers=2,
                                bump=sw.BUMP_QG, ctx=ctx)
        U0 = model.max_speed()
        loop = sw.TwoLayerLoop(model, ens, 0.25 * (L / nx) / U0, U0, 0.25, 0.0, nsub=5, speculate=speculate,
                               integrator=integrator)
        for _ in range(20):
            loop.step()
        loop.flush()
        ctx.synchronize()
        # TwoLayerLoop.step with every call timed (same calls, same order)
        names = ("cfl", "resolve", "snapshot", "packets", "speculate", "U0 result")
        acc = dict.fromkeys(names, 0.0)
        t_start = time.perf_counter()
        for _ in range(steps):
            t = time.perf_counter()
            loop.steps += 1
            loop.dt, changed = model.cfl_rule(loop.dt, loop.U0, loop.cfl_fraction)
            loop.dts.append(loop.dt)
            t1 = time.perf_counter(); acc["cfl"] += t1 - t; t = t1
            if model.spec_pending:
                model.resolve(not changed)
                if changed:
                    model.step(loop.dt)
                    model.max_speed_async()
            else:
                model.step(loop.dt)
                model.max_speed_async()
            loop.t = loop.t + loop.dt
            t1 = time.perf_counter(); acc["resolve"] += t1 - t; t = t1
            ny = 2 * nx
            if not loop.have_cur:
                model.snapshot(0, which=1, layer=0, ny_period=ny)
            model.snapshot(loop.group.next_slot(), which=0, layer=0, ny_period=ny)
            loop.have_cur = True
            t1 = time.perf_counter(); acc["snapshot"] += t1 - t; t = t1
            early = speculate and integrator == "ode23"
            if early:
                model.step_speculative(loop.dt)
                t1 = time.perf_counter(); acc["speculate"] += t1 - t; t = t1
            loop.group.add(loop.dt)
            t1 = time.perf_counter(); acc["packets"] += t1 - t; t = t1
            if speculate and not early:
                model.step_speculative(loop.dt)
                t1 = time.perf_counter(); acc["speculate"] += t1 - t; t = t1
            loop.U0 = model.max_speed_result()
            t1 = time.perf_counter(); acc["U0 result"] += t1 - t
        loop.flush()
        ctx.synchronize()
        wall = (time.perf_counter() - t_start) / steps * 1e6
        loop.settle()
        parts = "  ".join(f"{n} {acc[n] / steps * 1e6:.1f}" for n in names)
        print(f"{integrator} nx={nx} N={N}: {wall:.1f} us per driver step; host per call (us): {parts}", flush=True)
    finally:
        ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--integrator", choices=["leapfrog", "ode23"], default="leapfrog")
    args = ap.parse_args()
    for nx, N in ((64, 1000), (512, 125_000), (512, 1_000_000)):
        run(nx, N, args.steps, integrator=args.integrator)


if __name__ == "__main__":
    main()
