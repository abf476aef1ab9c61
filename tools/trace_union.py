"""Busy time of the packet kernel in a rocprofv3 kernel trace (diagnostic).

With two packet streams every launch is two half launches that overlap the
neighbouring calls', so the kernel-stats average (one half's duration) is not
the time a launch occupies the GPU.  This prints, over the trace's
tile_leapfrog_kernel dispatches: the half-launch average, the union of all
their busy intervals, and that union per launch (pairs of halves) — the
figure bench.py's wall-time roofline basis bounds from above.
usage: python tools/trace_union.py <kernel_trace.csv> [--last N]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="tile_leapfrog_kernel")
    ap.add_argument("--last", type=int, default=0, help="only the last N dispatches (the timed phase)")
    args = ap.parse_args()
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"])
    if args.last:
        iv = iv[-args.last:]
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    n = len(iv)
    print(f"dispatches {n}  mean dispatch {sum(e - s for s, e in iv) / n / 1e3:.1f} us  "
          f"union {busy / 1e3:.1f} us over a span of {span / 1e3:.1f} us  "
          f"union per launch pair {busy / (n / 2) / 1e3:.1f} us  busy share {busy / span:.3f}")


if __name__ == "__main__":
    main()
