"""Diagnostic: per-workgroup phase timeline of the tile kernel.

Needs a -DSWRT_PHASE_TIMING build (tools/sweep builds it as
build/variants/phase.so) passed through SWRT_LIB_PATH.  Runs the bench
workload, then for a few single steps reads the per-tile stamps
(s_memrealtime, 100 MHz) and prints phase shares, per-CU residency and the
spread of workgroup start times.  Read SHARES, not absolute time: the stamp
build's barriers-plus-stamps differ from the product kernel."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import swraytracing_amd as sw  # noqa: E402
from swraytracing_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=512)
    ap.add_argument("--packets", type=int, default=1_000_000)
    ap.add_argument("--mode", default="blend")
    ap.add_argument("--samples", type=int, default=5)
    ap.add_argument("--substeps", type=int, default=5)
    ap.add_argument("--rebin-every", type=int, default=20)
    ap.add_argument("--streams", type=int, default=1,
                    help="packet streams (1: the stamps are indexed by blockIdx, which two part launches share)")
    ap.add_argument("--dump", default="", help="save every sample's raw stamps (npz) for offline analysis")
    args = ap.parse_args()
    args.world, args.rank, args.seed = 1, 0, 146
    lib = _lib.load()
    f = lib.swrt_debug_phases
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    ctx = sw.Context(0)
    ctx.set_locality(args.rebin_every, 0)
    ctx.set_kernel(2)
    ctx.set_packet_streams(args.streams)
    bench._imports()
    w = bench.build_workload(ctx, args, 0, args.packets, args.packets)
    ctx.packets_set(w["x"], w["k"])
    for _ in range(8):
        bench.step(ctx, w, args.substeps)
    ntiles = (args.nx // 16) ** 2
    nrows = 4 * ntiles  # workgroups
    buf = np.zeros(nrows * 8, dtype=np.uint64)
    ptr = buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong))
    res = []
    raw = []
    for s in range(args.samples):
        assert f(None, nrows, 1) == 0
        bench.step(ctx, w, args.substeps)
        ctx.synchronize()
        assert f(ptr, nrows, 0) == 0
        d = buf.reshape(nrows, 8).astype(np.int64)
        d = d[d[:, 0] != 0]
        raw.append(d.copy())
        # word 6: packets of the tile | the SIMD id of every wave (2 bits each) << 32
        d[:, 6] &= 0xFFFFFFFF
        t0 = d[:, 0].min()
        P = (d[:, :5] - t0) * 10.0 / 1e3  # us
        stage = P[:, 1] - P[:, 0]
        sort = P[:, 2] - P[:, 1]
        comp = P[:, 3] - P[:, 2]
        tail = P[:, 4] - P[:, 3]
        life = P[:, 4] - P[:, 0]
        span = P[:, 4].max()
        hw = d[:, 7] & 0xFFFFFFFF
        xcc = d[:, 7] >> 32
        cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
        ucu = np.unique(cu)
        per_cu = np.array([np.sum(cu == c) for c in ucu])
        # busy fraction of each CU: union of its workgroups' lifetimes / span
        busy = []
        for c in ucu:
            iv = sorted(zip(P[cu == c, 0], P[cu == c, 4]))
            tot, cur_s, cur_e = 0.0, None, None
            for a_, b_ in iv:
                if cur_e is None or a_ > cur_e:
                    if cur_e is not None:
                        tot += cur_e - cur_s
                    cur_s, cur_e = a_, b_
                else:
                    cur_e = max(cur_e, b_)
            tot += cur_e - cur_s
            busy.append(tot / span)
        res.append(dict(
            span_us=float(span),
            wg_life_us_median=float(np.median(life)),
            share_stage=float(stage.sum() / life.sum()), share_sort=float(sort.sum() / life.sum()),
            share_compute=float(comp.sum() / life.sum()), share_tail=float(tail.sum() / life.sum()),
            stage_us_median=float(np.median(stage)), sort_us_median=float(np.median(sort)),
            compute_us_median=float(np.median(comp)), tail_us_median=float(np.median(tail)),
            compute_us_p90=float(np.percentile(comp, 90)),
            start_us_p50=float(np.median(P[:, 0])), start_us_max=float(P[:, 0].max()),
            end_us_min=float(P[:, 4].min()),
            cus=int(len(ucu)), wg_per_cu_min=int(per_cu.min()), wg_per_cu_max=int(per_cu.max()),
            cu_busy_mean=float(np.mean(busy)), cu_busy_min=float(np.min(busy)),
            packets_per_tile_mean=float(d[:, 6].mean()), packets_per_tile_max=int(d[:, 6].max()),
            mean_concurrent_wg=float(life.sum() / span),
            # first-round workgroups (start within 2 us) vs the rest
            compute_us_round1=float(np.median(comp[P[:, 0] < 2.0])) if np.any(P[:, 0] < 2.0) else None,
            compute_us_later=float(np.median(comp[P[:, 0] >= 2.0])) if np.any(P[:, 0] >= 2.0) else None,
            stage_us_round1=float(np.median(stage[P[:, 0] < 2.0])) if np.any(P[:, 0] < 2.0) else None,
            stage_us_later=float(np.median(stage[P[:, 0] >= 2.0])) if np.any(P[:, 0] >= 2.0) else None,
            n_round1=int(np.sum(P[:, 0] < 2.0)),
            corr_compute_packets=float(np.corrcoef(comp, d[:, 6])[0, 1]),
            compute_us_by_packets={f"{lo}-{lo + 64}": float(np.median(comp[(d[:, 6] >= lo) & (d[:, 6] < lo + 64)]))
                                   for lo in range(0, 1152, 64) if np.any((d[:, 6] >= lo) & (d[:, 6] < lo + 64))},
            compute_us_deciles=[float(v) for v in np.percentile(comp, np.arange(0, 101, 10))],
            compute_us_by_xcc={int(x): float(np.median(comp[xcc == x])) for x in np.unique(xcc)},
            compute_us_round1_by_xcc={int(x): float(np.median(comp[(xcc == x) & (P[:, 0] < 2.0)]))
                                      for x in np.unique(xcc) if np.any((xcc == x) & (P[:, 0] < 2.0))},
            slow_share_by_xcc={int(x): float(np.mean(comp[xcc == x] > 24.0)) for x in np.unique(xcc)},
            slow_share_by_tile_row_band={int(b): float(np.mean(comp[(np.arange(len(comp)) // 32) // 4 == b] > 24.0))
                                         for b in range(8)},
            fallback_per_tile_mean=float(d[:, 5].mean()), fallback_per_tile_max=int(d[:, 5].max()),
            corr_compute_fallback=float(np.corrcoef(comp, d[:, 5])[0, 1]),
            compute_us_by_fallback={f"{lo}-{hi}": [float(np.median(comp[(d[:, 5] >= lo) & (d[:, 5] < hi)])),
                                                   int(np.sum((d[:, 5] >= lo) & (d[:, 5] < hi)))]
                                    for lo, hi in [(0, 1), (1, 5), (5, 20), (20, 50), (50, 100), (100, 100000)]
                                    if np.any((d[:, 5] >= lo) & (d[:, 5] < hi))},
        ))
    print(json.dumps(res[-1], indent=1))
    if args.dump:
        np.savez_compressed(args.dump, stamps=np.stack(raw))
    print(json.dumps({"span_us_all": [r["span_us"] for r in res]}))
    ctx.close()


if __name__ == "__main__":
    main()
