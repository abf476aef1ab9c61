"""Where the wall time of a bench run goes: reads a rocprofv3 kernel trace
(`--kernel-trace --output-format csv`) and, over the last `--launches` packet
launches, reports the GPU busy time per kernel and the idle gaps between
kernels (launch latency, host work, synchronisation).
usage: python tools/timeline.py <run>_kernel_trace.csv [--launches 50]"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--match", default="leapfrog")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    hot = [i for i, r in enumerate(rows) if args.match in r["Kernel_Name"]]
    if len(hot) < args.launches + 1:
        raise SystemExit(f"only {len(hot)} '{args.match}' launches in the trace")
    first, last = hot[-args.launches], hot[-1]
    seg = rows[first:last + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = int(seg[-1]["End_Timestamp"])
    busy = collections.defaultdict(float)
    calls = collections.Counter()
    gaps = []
    prev_end = None
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        busy[name] += (e - s) / 1e3
        calls[name] += 1
        if prev_end is not None:
            gaps.append((s - prev_end) / 1e3)
        prev_end = max(prev_end or 0, e)
    span = (t1 - t0) / 1e3
    out = {"launches": args.launches, "span_us": span, "per_launch_us": span / args.launches,
           "gpu_busy_us": {k: round(v, 1) for k, v in sorted(busy.items(), key=lambda kv: -kv[1])},
           "calls": dict(calls),
           "gap_total_us": round(sum(g for g in gaps if g > 0), 1),
           "gap_max_us": round(max(gaps), 1) if gaps else 0.0,
           "gap_median_us": round(sorted(gaps)[len(gaps) // 2], 2) if gaps else 0.0}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
