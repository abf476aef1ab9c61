"""Host time between the drivers' ode23 intervals (diagnostic).

Runs TwoLayerLoop with integrator="ode23" on the bench workload (512^2 x 2,
1e6 packets by default) and wraps the context's calls with host timers: the
time from one swrt_ode23_run_hooked return to the next call, split by the
calls made in between, and the wall time of each ode23 call.  While the
library's controller waits for the interval's last attempt the GPU is busy;
from that return to the next call's first launch it idles, so this gap is
what an interval pays on top of its launches.
usage: python tools/ode23_host_gap.py [--packets N] [--steps K]"""
import argparse
import collections
import json
import math
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import swraytracing_amd as sw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=12)
    args = ap.parse_args()
    a = bench.parse_args(["--packets", str(args.packets)])
    a.world, a.rank = 1, 0
    bench._imports()
    ctx = sw.Context(0)
    w = bench.build_workload(ctx, a, 0, args.packets, args.packets)
    nx, L, f, Cg = w["nx"], w["L"], w["f"], math.sqrt(w["gH"])
    qk = np.stack([w["qk1"], -w["qk1"]], axis=2)
    model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
    ens = sw.PacketEnsemble(w["x"], w["k"], L, f, Cg, nx, f / Cg, shear=0.5, k_scale=2 * math.pi / L, nlayers=2,
                            bump=sw.BUMP_QG, ctx=ctx)
    U0 = model.max_speed()
    loop = sw.TwoLayerLoop(model, ens, 0.25 * (L / nx) / U0, U0, 0.25, 0.0, nsub=5, integrator="ode23")
    for _ in range(4):
        loop.step()
    ctx.synchronize()
    # host timers around every context call
    acc = collections.defaultdict(float)
    cnt = collections.Counter()
    state = {"last_ret": None, "gap": [], "in_gap": collections.defaultdict(float), "run": []}
    names = [n for n in dir(ctx) if not n.startswith("_") and callable(getattr(ctx, n))]
    for n in names:
        fn = getattr(ctx, n)

        def wrap(fn=fn, n=n):
            def inner(*aa, **kk):
                t0 = time.perf_counter()
                if n == "ode23_run" and state["last_ret"] is not None:
                    state["gap"].append(t0 - state["last_ret"])
                r = fn(*aa, **kk)
                t1 = time.perf_counter()
                acc[n] += t1 - t0
                cnt[n] += 1
                if n == "ode23_run":
                    state["run"].append(t1 - t0)
                    state["last_ret"] = t1
                elif state["last_ret"] is not None:
                    state["in_gap"][n] += t1 - t0
                return r
            return inner
        setattr(ctx, n, wrap())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loop.step()
    loop.flush()
    ctx.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    gaps = np.array(state["gap"]) * 1e6
    out = {"packets": args.packets, "ms_per_step": wall * 1e3,
           "ode23_call_ms_median": float(np.median(state["run"]) * 1e3),
           "host_gap_us_median": float(np.median(gaps)), "host_gap_us": [round(g, 1) for g in gaps],
           "calls_in_gaps_us_per_gap": {k: round(v / max(1, len(gaps)) * 1e6, 1) for k, v in state["in_gap"].items()},
           "per_call_us": {k: round(acc[k] / cnt[k] * 1e6, 1) for k in cnt}}
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
