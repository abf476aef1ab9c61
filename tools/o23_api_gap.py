"""Host timeline between the drivers' ode23 intervals from a rocprofv3
--hip-runtime-trace --kernel-trace run (diagnostic; tools/sess_o23api.sh).

For every chained interval: the host time from the API call that launched the
interval's stage 1 (queued by the previous call as it ended) to the call that
launched its first-step kernel, the HIP calls in between grouped by name
(count and host time), and the GPU idle between stage 1's end and the first
step's start.  usage: python tools/o23_api_gap.py <trace dir>"""
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


def main(d):
    api = sorted(load(d, "*hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    ker = {r["Correlation_Id"]: r for r in load(d, "*kernel_trace.csv")}
    launches = []  # (api row, kernel row)
    for r in api:
        k = ker.get(r["Correlation_Id"])
        if k is not None:
            launches.append((r, k))
    out = []
    for i, (r, k) in enumerate(launches):
        if "tile_ode23_kernel<1" not in k["Kernel_Name"]:
            continue
        # the next first-step launch after this stage 1
        j = next((j for j in range(i + 1, len(launches)) if "ode23_first_step" in launches[j][1]["Kernel_Name"]), None)
        if j is None:
            continue
        r2, k2 = launches[j]
        t0, t1 = int(r["Start_Timestamp"]), int(r2["Start_Timestamp"])
        calls = collections.defaultdict(lambda: [0, 0.0])
        for a in api:
            s = int(a["Start_Timestamp"])
            if t0 < s < t1:
                c = calls[a["Function"]]
                c[0] += 1
                c[1] += (int(a["End_Timestamp"]) - s) / 1e3
        out.append({
            "host_us_stage1_to_first_step_launch": (t1 - t0) / 1e3,
            "stage1_gpu_us": (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3,
            "gpu_idle_us_stage1_end_to_first_step": (int(k2["Start_Timestamp"]) - int(k["End_Timestamp"])) / 1e3,
            "launch_to_start_us_first_step": (int(k2["Start_Timestamp"]) - t1) / 1e3,
            "calls": {n: [c[0], round(c[1], 1)] for n, c in sorted(calls.items(), key=lambda x: -x[1][1])},
        })
    for o in out:
        print(json.dumps(o))
    if out:
        med = lambda key: sorted(o[key] for o in out)[len(out) // 2]
        print(json.dumps({"intervals": len(out), **{f"median_{key}": med(key) for key in (
            "host_us_stage1_to_first_step_launch", "stage1_gpu_us", "gpu_idle_us_stage1_end_to_first_step",
            "launch_to_start_us_first_step")}}))


if __name__ == "__main__":
    main(sys.argv[1])
