"""What gates the leapfrog driver's packet launches: for each packet launch on
the packet stream's queue, the kernel (any queue) whose end most closely
precedes its start, counted by kernel and with the median gap.  Input: a
rocprofv3 `--kernel-trace --output-format csv` of `bench.py --driver-steps N`.
usage: python tools/lf_launch_gates.py <run>_kernel_trace.csv [--queue 1]"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--queue", default="1", help="Queue_Id of the packet stream")
    ap.add_argument("--max", type=int, default=300, help="launches analysed (from the middle third on)")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ends = sorted(rows, key=lambda r: int(r["End_Timestamp"]))
    launches = [r for r in rows if "tile_leapfrog" in r["Kernel_Name"] and r["Queue_Id"] == args.queue]
    launches = launches[len(launches) // 3:len(launches) // 3 + args.max]
    count = collections.Counter()
    gaps = collections.defaultdict(list)
    j = 0
    for launch in launches:
        s = int(launch["Start_Timestamp"])
        while j + 1 < len(ends) and int(ends[j + 1]["End_Timestamp"]) <= s:
            j += 1
        prev = ends[j]
        if int(prev["End_Timestamp"]) > s:
            continue
        name = prev["Kernel_Name"].split("(")[0].replace("void ", "")[-40:] + " q" + prev["Queue_Id"]
        count[name] += 1
        gaps[name].append((s - int(prev["End_Timestamp"])) / 1e3)
    for name, n in count.most_common():
        print(f"{n:5d}  {name:48s} median gap {statistics.median(gaps[name]):7.2f} us")


if __name__ == "__main__":
    main()
