"""Diagnostic: tile-kernel launch time by position in the re-binning cycle
(HIP events on every launch, one synchronising read per step)."""
import argparse
import json
import os
import sys

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import swraytracing_amd as sw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rebin-every", type=int, default=4)
    ap.add_argument("--cell-sort", type=int, default=0)
    ap.add_argument("--mode", default="blend")
    ap.add_argument("--steps", type=int, default=48)
    args = ap.parse_args()
    args.nx, args.packets, args.world, args.rank, args.seed = 512, 1_000_000, 1, 0, 146
    ctx = sw.Context(0)
    ctx.set_locality(args.rebin_every, 0)
    ctx.set_cell_sort(args.cell_sort)
    w = bench.build_workload(ctx, args, np.random.default_rng(146))
    ctx.packets_set(w["x"], w["k"])
    for _ in range(8):
        bench.step(ctx, w, 1)
    ctx.set_timing(1)
    ctx.kernel_time(reset=True)
    times = []
    for _ in range(args.steps):
        bench.step(ctx, w, 1)
        ms, n = ctx.kernel_time(reset=True)
        times.append(ms * 1e3 / max(n, 1))
    t = np.array(times)
    R = args.rebin_every
    by = {int(p): float(t[p::R].mean()) for p in range(R)}
    print(json.dumps({"rebin_every": R, "cell_sort": args.cell_sort, "mean_us": float(t.mean()),
                      "by_position_us": by}))
    ctx.close()


if __name__ == "__main__":
    main()
