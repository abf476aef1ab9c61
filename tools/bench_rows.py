"""Measurement of the SURVEY §8 rows beside the headline packet kernel (A10
step_packet_xka, A12 omega histogram, A5/A8/A9 field preparation) on one
GPU.  Prints one JSON line; not the driver's bench (bench.py is).

  xka        swrt_xka_step (ray_trace_sw/step_packet_xka.m: RK4 in x, k and
             the action a, 15 stencil interpolations with cg_sw per tap) on a
             256^2 Childress-Soward background (raytrace.m:30-37) with a
             smooth H, 1e6 packets; per-step device time from the difference
             of a 60- and a 10-step call (the host copies cancel)
  histogram  swrt_omega_histogram (analysis/load_data.m:33-52) of 1e6
             device-resident packets, 100 bins
  field_qk   swrt_set_field_qk at 512^2 (grid_U.m: 2 MB host spectrum in,
             6 derivative fields out, GPU FFTs), per snapshot
"""
import json
import math
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import swraytracing_amd as sw  # noqa: E402


def wall(ctx, fn, reps):
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ctx = sw.Context(0)
    rng = np.random.default_rng(3)
    out = {}

    # --- A10 step_packet_xka: 256^2 cellular flow (raytrace.m:30-37) + smooth H
    nx, L = 256, 2 * math.pi
    xg = np.arange(nx) * (L / nx)
    X, Y = np.meshgrid(xg, xg, indexing="ij")
    U0, km, a = 0.1, 4.0, 0.25
    s, c = np.sin, np.cos
    U = {"u": -U0 * (s(km * X) * c(km * Y) - a * c(km * X) * s(km * Y)),
         "v": U0 * (c(km * X) * s(km * Y) - a * s(km * X) * c(km * Y))}
    G = {"u_x": -km * U0 * (c(km * X) * c(km * Y) + a * s(km * X) * s(km * Y)),
         "u_y": km * U0 * (s(km * X) * s(km * Y) + a * c(km * X) * c(km * Y)),
         "v_x": -km * U0 * (s(km * X) * s(km * Y) + a * c(km * X) * c(km * Y)),
         "v_y": km * U0 * (c(km * X) * c(km * Y) + a * s(km * X) * s(km * Y))}
    H = 1.0 + 0.1 * np.cos(2 * X + Y) + 0.05 * np.sin(3 * Y)
    dx = L / nx
    ctx.xka_set_fields(U, G, H, dx, dx)
    N = 1_000_000
    th = rng.random(N) * 2 * np.pi
    st = np.stack([rng.random(N) * L, rng.random(N) * L, 3 * np.cos(th), 3 * np.sin(th), np.ones(N)], axis=1)
    dt = 0.05 * dx / U0
    ctx.xka_step(st, 1.0, 1.0, dt, 2)  # warm-up
    t10 = wall(ctx, lambda: ctx.xka_step(st, 1.0, 1.0, dt, 10), 2)
    t60 = wall(ctx, lambda: ctx.xka_step(st, 1.0, 1.0, dt, 60), 2)
    per_step = (t60 - t10) / 50
    out["xka"] = {"nx": nx, "packets": N, "us_per_step": per_step * 1e6,
                  "packet_steps_per_s": N / per_step,
                  "call_10_steps_ms": t10 * 1e3, "note": "RK4 x/k/a, 15 interpolations per packet-step"}

    # --- A12 omega histogram of device-resident packets
    x = (rng.random((N, 2)) - 0.5) * 20.0
    k = 3.0 * np.sqrt(15.0) * np.stack([np.cos(th), np.sin(th)], axis=1) * (1 + 0.1 * rng.random((N, 1)))
    ctx.packets_set(x, k)
    edges = np.linspace(3.0, 20.0, 101)
    ctx.omega_histogram(3.0, 1.0, edges)
    th_ = wall(ctx, lambda: ctx.omega_histogram(3.0, 1.0, edges), 20)
    out["omega_histogram"] = {"packets": N, "bins": 100, "us_per_call": th_ * 1e6,
                              "packets_per_s": N / th_, "note": "includes the 100-bin count read-back"}

    # --- A5/A8/A9 field preparation (grid_U on the GPU) at 512^2
    nx = 512
    kmax = nx // 2 - 1
    qk = np.zeros((2 * kmax + 1, kmax + 1), complex)
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(kmax + 1)[None, :]
    ring = (kx * kx + ky * ky > 100) & (kx * kx + ky * ky <= 900)
    qk[ring] = np.exp(2j * np.pi * rng.random(ring.sum())) * 0.01
    ctx.set_field_qk(0, qk, nx, 20.0, 3.0, 0.5, 2 * np.pi / 20.0, 2 * nx)
    tq = wall(ctx, lambda: ctx.set_field_qk(0, qk, nx, 20.0, 3.0, 0.5, 2 * np.pi / 20.0, 2 * nx), 10)
    out["field_qk"] = {"nx": nx, "ms_per_snapshot": tq * 1e3,
                       "note": "host spectrum upload + 6 derivative spectra + 3 packed inverse 2-D FFTs + pack"}
    ctx.close()
    print(json.dumps({"metric": "SURVEY 8 rows beside the packet kernel (1 x MI355X)", **out}))


if __name__ == "__main__":
    main()
