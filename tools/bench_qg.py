"""The 2-layer QG PDE alone (no packets): the qg2layersw_raytrace loop's
device work per PDE step — AB3 update, the fused post-step transforms
(Jacobian inputs, CFL speed, layer 0's grid_U) and the snapshot pack — for
per-kernel counters (tools/pmc_qg.sh).  512^2 x 2 layers by default.
Prints one JSON line with the mean step time."""
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
from swraytracing_amd.qg import initial_q  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=512)
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    nx, L, f, Cg = args.nx, 20.0, 3.0, 1.0
    ctx = sw.Context(0)
    rng = np.random.default_rng(5)
    q1 = initial_q(nx, L, 0.2, f / Cg, 10, 30, rng, ndgrid=True)
    qk = np.stack([ctx.g2k(q1), ctx.g2k(-q1)], axis=2)
    model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
    dt = 0.25 * (L / nx) / model.max_speed()
    for _ in range(4):
        model.step(dt)
        model.snapshot(1, which=0, ny_period=2 * nx)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        model.step(dt)
        model.max_speed_async()
        model.snapshot(1, which=0, ny_period=2 * nx)
        model.max_speed_result()
    ctx.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    print(json.dumps({"what": "2-layer QG PDE step + CFL speed + snapshot, no packets", "nx": nx,
                      "ms_per_step": ms, "dt": dt, "finite": bool(np.isfinite(model.qk).all())}))
    ctx.close()


if __name__ == "__main__":
    main()
