"""Driver-step anatomy from a rocprofv3 kernel trace of bench.py's
driver_step phase (diagnostic): per QG kernel its median duration while the
packets run beside it (the last --steps driver steps), the QG chain per step
(update start -> U0 copy end), and the packet launches' span per step.
usage: python tools/driver_trace_summary.py <kernel_trace.csv> [--steps 40]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--timeline", type=int, default=0,
                    help="also print every kernel of the last N steps: start/end (us from the step's update), stream")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    upd = [i for i, r in enumerate(rows) if "qg_update_kernel" in r["Kernel_Name"]]
    seg = rows[upd[-args.steps - 1]:upd[-1]]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["Start_Timestamp"])
    dur = collections.defaultdict(list)
    for r in seg:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "leapfrog" in name:
            name = "tile_leapfrog_kernel (half launch)"
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{args.steps} driver steps, {(t1 - t0) / args.steps / 1e3:.1f} us per step (update to update)")
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"  {name[:48]:48s} n={len(v):4d} median {v[len(v) // 2]:7.1f} us  total/step {sum(v) / args.steps:7.1f} us")
    chain, st = [], None
    for r in seg:
        if "qg_update_kernel" in r["Kernel_Name"]:
            st = int(r["Start_Timestamp"])
        if "copyBuffer" in r["Kernel_Name"] and st is not None:
            chain.append((int(r["End_Timestamp"]) - st) / 1e3)
            st = None
    chain.sort()
    if chain:
        print(f"  QG chain update -> U0 copy: median {chain[len(chain) // 2]:.1f} us")
    if args.timeline:
        tl = rows[upd[-args.timeline - 1]:upd[-1]]
        z = int(tl[0]["Start_Timestamp"])
        busy = 0
        for r in tl:
            a, b = (int(r["Start_Timestamp"]) - z) / 1e3, (int(r["End_Timestamp"]) - z) / 1e3
            print(f"  {a:8.1f} {b:8.1f} {b - a:7.1f}  q{r['Queue_Id']:>3s} s{r['Stream_Id']:>3s}  "
                  f"{r['Kernel_Name'].split('(')[0].replace('void ', '')[:60]}")


if __name__ == "__main__":
    main()
