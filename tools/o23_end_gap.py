"""The host's HIP calls at the end of the drivers' ode23 intervals, from a
rocprofv3 --hip-runtime-trace --kernel-trace run (diagnostic;
tools/sess_o23end.sh).

For every interval end: the time the last attempt's kernels finished (both
parts), then every HIP call from then until the call that launched the next
kernel on the packet stream's queue (the chain's re-binning or stage 1), with
its start relative to that end and its host duration; then the GPU idle until
that kernel started.  usage: python tools/o23_end_gap.py <trace dir> [--show N]"""
import argparse
import collections
import csv
import glob
import json
import os
import sys


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not f:
        sys.exit(f"no {pat} under {d}")
    return list(csv.DictReader(open(f[0])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--show", type=int, default=3, help="interval ends printed call by call")
    args = ap.parse_args()
    api = sorted(load(args.trace_dir, "*hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    kers = sorted(load(args.trace_dir, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    launch_of = {}
    for r in api:
        launch_of.setdefault(r["Correlation_Id"], r)
    ends = []
    for i, k in enumerate(kers):
        if "tile_ode23_kernel<1," not in k["Kernel_Name"]:
            continue
        # the previous attempt kernels (stage 0): the last two before this point
        prev = [r for r in kers[max(0, i - 12):i] if "tile_ode23_kernel<0," in r["Kernel_Name"]]
        if len(prev) < 2:
            continue
        t_end = max(int(r["End_Timestamp"]) for r in prev[-2:])
        # the first kernel after the attempts (re-binning or stage 1)
        nxt = [r for r in kers[max(0, i - 12):i + 1] if int(r["Start_Timestamp"]) >= t_end]
        first = nxt[0] if nxt else k
        la = launch_of.get(first["Correlation_Id"])
        if la is None:
            continue
        t_launch = int(la["Start_Timestamp"])
        calls = [r for r in api if t_end - 2000 <= int(r["Start_Timestamp"]) <= t_launch]
        ends.append({
            "gpu_idle_us": round((int(first["Start_Timestamp"]) - t_end) / 1e3, 1),
            "host_end_to_launch_us": round((t_launch - t_end) / 1e3, 1),
            "first_kernel": first["Kernel_Name"][:40],
            "calls": [(r["Function"] if "Function" in r else r.get("Operation", "?"),
                       round((int(r["Start_Timestamp"]) - t_end) / 1e3, 1),
                       round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1)) for r in calls],
        })
    for e in ends[-args.show:]:
        print(json.dumps({k: v for k, v in e.items() if k != "calls"}))
        for name, s, d in e["calls"]:
            print(f"    {s:8.1f} {d:7.1f}  {name}")
    agg = collections.Counter()
    for e in ends:
        for name, _, d in e["calls"]:
            agg[name] += d
    n = max(1, len(ends))
    print(json.dumps({"intervals": len(ends),
                      "mean_gpu_idle_us": round(sum(e["gpu_idle_us"] for e in ends) / n, 1),
                      "mean_host_end_to_launch_us": round(sum(e["host_end_to_launch_us"] for e in ends) / n, 1),
                      "host_us_per_interval_by_call": {k: round(v / n, 1) for k, v in agg.most_common()}}))


if __name__ == "__main__":
    main()
