"""Launch-gap probe: the bench's packet loop (configs[3] workload) with the
context's per-call stream events on or off (swrt_qg_set_stream: the QG
stream's slot events) and with or without sampled HIP-event timing, so a
rocprofv3 kernel trace shows what sits between two dependent packet
launches.  usage: python tools/gap_probe.py [--one-stream] [--timing-every K] [--steps S]"""
import argparse
import os
import sys
import time

import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import swraytracing_amd as sw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--one-stream", action="store_true")
    ap.add_argument("--timing-every", type=int, default=0)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    args = argparse.Namespace(nx=512, packets=1_000_000, substeps=5, rebin_every=20, tile=0, mode="blend",
                              positions="uniform", seed=0, intervals=1, world=1, rank=0)
    ctx = sw.Context(0)
    if a.one_stream:
        ctx.qg_set_stream(0)
    ctx.set_locality(args.rebin_every, args.tile)
    w = bench.build_workload(ctx, args, np.random.default_rng(0))
    ctx.packets_set(w["x"], w["k"])
    for _ in range(8):
        bench.step(ctx, w, args.substeps)
    ctx.synchronize()
    ctx.set_timing(a.timing_every)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        bench.step(ctx, w, args.substeps)
    ctx.synchronize()
    el = time.perf_counter() - t0
    print(f"one_stream={a.one_stream} timing_every={a.timing_every}: {el / a.steps * 1e3:.4f} ms per step, "
          f"{args.packets * args.substeps * a.steps / el:.4g} packet-steps/s")


if __name__ == "__main__":
    main()
