"""Host/device timeline of bench.py's driver steps (diagnostic): a rocprofv3
run with --kernel-trace --hip-trace gives each kernel's dispatch API call
(matched by Correlation_Id) and the host's blocking calls, so the gaps in the
device timeline can be told apart: a kernel that starts long after the
previous one on its queue ended either was queued late (host) or waited on
another queue (event).
usage: python tools/driver_host_timeline.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv> [--steps 3]"""
import argparse
import csv
import glob
import os

BLOCKING = ("hipEventSynchronize", "hipStreamSynchronize", "hipDeviceSynchronize", "hipMemcpy", "hipMalloc",
            "hipFree", "hipHostMalloc", "hipMemcpyDtoH", "hipMemcpyHtoD", "hipEventQuery")


def load(pattern):
    f = glob.glob(pattern, recursive=True)
    if not f:
        raise SystemExit(f"no file {pattern}")
    return list(csv.DictReader(open(f[0])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    ker = sorted(load(os.path.join(args.dir, "**", "*kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
    api = load(os.path.join(args.dir, "**", "*hip_api_trace.csv"))
    by_corr = {r["Correlation_Id"]: r for r in api}
    upd = [i for i, r in enumerate(ker) if "qg_update_kernel" in r["Kernel_Name"]]
    seg = ker[upd[-args.steps - 1]:upd[-1]]
    z = int(seg[0]["Start_Timestamp"])
    t_end = int(seg[-1]["End_Timestamp"])
    ev = []
    for r in seg:
        a = by_corr.get(r["Correlation_Id"])
        q = (int(a["Start_Timestamp"]) - z) / 1e3 if a else float("nan")
        ev.append((int(r["Start_Timestamp"]), "K", q, (int(r["Start_Timestamp"]) - z) / 1e3,
                   (int(r["End_Timestamp"]) - z) / 1e3, f"q{r['Queue_Id']}",
                   r["Kernel_Name"].split("(")[0].replace("void ", "")[:56]))
    for a in api:
        s, e = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
        if e < z or s > t_end:
            continue
        fn = a.get("Function") or a.get("Operation") or ""
        if any(fn.startswith(b) for b in BLOCKING) and e - s > 2000:
            ev.append((s, "H", (s - z) / 1e3, (s - z) / 1e3, (e - z) / 1e3, "host", fn))
    ev.sort()
    print("  kind  queued    start      end    dur  where  what")
    for _, kind, q, a, b, where, what in ev:
        print(f"  {kind:4s} {q:8.1f} {a:8.1f} {b:8.1f} {b - a:6.1f}  {where:5s}  {what}")


if __name__ == "__main__":
    main()
