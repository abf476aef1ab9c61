"""One ode23 driver interval from a rocprofv3 kernel trace (`--kernel-trace
--output-format csv` of `bench.py --ode23-steps K`): every kernel between two
consecutive stage-1 launches (tile_ode23_kernel<1, ...>), with its queue,
start relative to the stage-1 launch and duration, then the GPU idle time
(no kernel on any queue) per interval and where it falls.
usage: python tools/ode23_timeline.py <run>_kernel_trace.csv [--interval -2]"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--interval", type=int, default=-2, help="which interval (python index over the trace's)")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    f1 = [i for i, r in enumerate(rows) if "tile_ode23_kernel<1," in r["Kernel_Name"]]
    if len(f1) < 3:
        raise SystemExit(f"only {len(f1)} stage-1 launches in the trace")
    spans = list(zip(f1[:-1], f1[1:]))
    a, b = spans[args.interval]
    t0 = int(rows[a]["Start_Timestamp"])
    lines = []
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("void ", "")[:60]
        lines.append(f"{name:60s} q{r.get('Queue_Id', '?'):>3s} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}")
    print("kernel | queue | start us | dur us (relative to the interval's stage-1 launch)")
    print("\n".join(lines))
    # idle: union of busy intervals over every queue, per interval
    out = []
    for a, b in spans:
        seg = rows[a:b + 1]
        t_start, t_end = int(seg[0]["Start_Timestamp"]), int(seg[-1]["Start_Timestamp"])
        busy_end = t_start
        idle = []
        for r in seg[:-1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s > busy_end:
                idle.append(((busy_end - t_start) / 1e3, (s - busy_end) / 1e3))
            busy_end = max(busy_end, e)
        if t_end > busy_end:
            idle.append(((busy_end - t_start) / 1e3, (t_end - busy_end) / 1e3))
        out.append({"interval_us": (t_end - t_start) / 1e3,
                    "idle_us": round(sum(d for _, d in idle), 1),
                    "idle_gaps_over_2us": [(round(s, 1), round(d, 1)) for s, d in idle if d > 2]})
    for o in out:
        print(json.dumps(o))
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
