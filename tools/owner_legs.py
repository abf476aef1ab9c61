"""Diagnostic: the two legs of the PDE-owner driver on one GPU (bench.py
owner_forecast), with the host time of every call of a step, to find what
bounds each leg.  usage: python tools/owner_legs.py [--receiver N ...] [--owner N ...]"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Timed:
    """Wraps a callable; accumulates its host time under `name`."""

    def __init__(self, acc, name, fn):
        self.acc, self.name, self.fn = acc, name, fn

    def __call__(self, *a, **k):
        t = time.perf_counter()
        try:
            return self.fn(*a, **k)
        finally:
            self.acc[self.name] = self.acc.get(self.name, 0.0) + time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--receiver", type=int, nargs="*", default=[142857])
    ap.add_argument("--owner", type=int, nargs="*", default=[0, 76923, 142857])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--ahead", type=int, default=None)
    ap.add_argument("--nbuf", type=int, default=5)
    ap.add_argument("--recv-qg-stream", type=int, default=0, help="receiver legs: snapshots on the QG stream (1)")
    ap.add_argument("--recv-streams", type=int, default=1, help="receiver legs: packet streams (1 or 2)")
    ap.add_argument("--owner-export", choices=["link", "packet", "none"], default="packet",
                    help="owner legs: the link on a torch stream of its own, on the packet stream (the driver's, "
                         "OwnerLink.bind_owner), or no export at all")
    ap.add_argument("--micro", type=int, nargs="*", default=[],
                    help="packet counts: time snapshot_qk alone, the packet interval alone, and both, back to back")
    a = ap.parse_args()
    import bench
    bench._imports()
    import torch

    import swraytracing_amd as sw
    args = bench.parse_args([])
    args.world, args.rank = 1, 0
    dev = torch.device("cuda", 0)
    ctx = sw.Context(0)
    w = bench.build_workload(ctx, args, 0, 1_000_000, 1_000_000)
    ctx.set_timing(0)  # (as the drivers)
    OneGPU = bench._owner_links()
    nx, L, f, Cg = w["nx"], w["L"], w["f"], math.sqrt(w["gH"])
    qk = np.stack([w["qk1"], -w["qk1"]], axis=2)
    out = {}

    def ensemble(n):
        return sw.PacketEnsemble(w["x"][:n], w["k"][:n], L, f, Cg, nx, f / Cg, shear=0.5, k_scale=2 * math.pi / L,
                                 nlayers=2, bump=sw.BUMP_QG, ctx=ctx)

    def run(loop, acc):
        for _ in range(30):
            loop.step()
        loop.flush()
        ctx.synchronize()
        torch.cuda.synchronize(dev)
        acc.clear()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            loop.step()
        loop.flush()
        ctx.synchronize()
        torch.cuda.synchronize(dev)
        el = (time.perf_counter() - t0) / a.steps * 1e3
        return el, {k: v / a.steps * 1e3 for k, v in acc.items()}

    for nr in a.micro:
        ctx.qg_set_stream(bool(a.recv_qg_stream))
        ctx.set_packet_streams(a.recv_streams)
        model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
        dt = 0.25 * (L / nx) / model.max_speed()
        link = OneGPU(nx)
        for b in link.bufs:
            link._export(ctx, b, dt)
        ens = ensemble(nr)
        ens.ctx.snapshot_qk(0, link.bufs[0].data_ptr(), nx, L, f / Cg, 0.5, 2 * math.pi / L, 2 * nx,
                            stream=link.stream.cuda_stream)

        def snap():
            ctx.snapshot_qk(1, link.bufs[0].data_ptr(), nx, L, f / Cg, 0.5, 2 * math.pi / L, 2 * nx)

        def adv():
            ens.advance_intervals([dt], 5)

        def snap_ev():
            ctx.snapshot_qk(1, link.bufs[0].data_ptr(), nx, L, f / Cg, 0.5, 2 * math.pi / L, 2 * nx,
                            stream=link.stream.cuda_stream)

        def swap():
            ctx.swap_slots(0, 1)

        res = {}
        for name, fns in (("snapshot", [snap]), ("packets", [adv]), ("both", [snap, adv]),
                          ("snapshot_ev", [snap_ev]), ("both_ev", [snap_ev, adv]), ("both_swap", [snap, adv, swap]),
                          ("both_ev_swap", [snap_ev, adv, swap])):
            for rep in range(2):
                ctx.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    for fn in fns:
                        fn()
                ctx.synchronize()
                res[name] = (time.perf_counter() - t0) / a.steps * 1e3
        print(f"micro {nr}: " + json.dumps({k: round(v, 4) for k, v in res.items()}), flush=True)
    for nr in a.receiver:
        ctx.qg_set_stream(bool(a.recv_qg_stream))
        ctx.set_packet_streams(a.recv_streams)
        model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
        dt = 0.25 * (L / nx) / model.max_speed()
        link = OneGPU(nx, dt, nbuf=a.nbuf)
        for b in link.bufs:
            link._export(ctx, b, dt)
        ens = ensemble(nr)
        loop = sw.ReceiverLoop(link, ens, dt, 0.0, nsub=5, ahead=a.ahead)
        acc = {}
        loop.step = Timed(acc, "step_total", loop.step)
        link.receive = Timed(acc, "receive", link.receive)
        link.snapshot = Timed(acc, "snapshot", link.snapshot)
        ens.advance_intervals = Timed(acc, "advance", ens.advance_intervals)
        ms, parts = run(loop, acc)
        out[f"receiver_{nr}"] = {"ms_per_step": ms, "host_ms": parts}
        print(f"receiver {nr}: {ms:.4f} ms/step, host {json.dumps({k: round(v, 4) for k, v in parts.items()})}",
              flush=True)
    ctx.qg_set_stream(True)
    ctx.set_packet_streams(2)
    for n0 in a.owner:
        model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
        U0 = model.max_speed()
        ens = ensemble(n0)
        link = OneGPU(nx)
        if a.owner_export == "packet":
            link.bind_owner(ctx)
        elif a.owner_export == "none":
            link.publish = lambda c_, dt: None
        loop = sw.TwoLayerLoop(model, ens, 0.25 * (L / nx) / U0, U0, 0.25, 0.0, nsub=5, link=link)
        acc = {}
        link.publish = Timed(acc, "publish", link.publish)
        for name in ("resolve", "step_speculative", "max_speed_result", "snapshot"):
            setattr(model, name, Timed(acc, name, getattr(model, name)))
        ens.advance_intervals = Timed(acc, "advance", ens.advance_intervals)
        ms, parts = run(loop, acc)
        loop.settle()
        out[f"owner_{n0}"] = {"ms_per_step": ms, "host_ms": parts}
        print(f"owner {n0}: {ms:.4f} ms/step, host {json.dumps({k: round(v, 4) for k, v in parts.items()})}",
              flush=True)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
