"""Parse rocprofv3 --pmc CSVs (FETCH_SIZE / WRITE_SIZE passes) into per-launch
HBM bytes of the leapfrog kernel; merge into profiles/traffic.json.

Units and gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md
§7): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced streaming read, so the read side is doubled
(`fetch_corrected`); the raw sum is kept beside it because the correction is
calibrated for 16-B/lane streaming reads only."""
import csv
import glob
import json
import os
import sys


def collect(d, counter):
    vals = []
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "leapfrog_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    d = sys.argv[1]
    args = sys.argv[2:]
    fetch = collect(d, "FETCH_SIZE")
    write = collect(d, "WRITE_SIZE")
    if not fetch or not write:
        print("no leapfrog_kernel rows found", file=sys.stderr)
        sys.exit(1)
    # skip warmup dispatches: use the median
    fetch.sort(); write.sort()
    f_kib = fetch[len(fetch) // 2]
    w_kib = write[len(write) // 2]
    raw = (f_kib + w_kib) * 1024.0
    corr = (2 * f_kib + w_kib) * 1024.0
    mode = "steady" if "--mode" in args and args[args.index("--mode") + 1] == "steady" else "blend"
    def arg(name, default):
        return int(args[args.index(name) + 1]) if name in args else default
    key = f"{mode}_nx{arg('--nx', 512)}_N{arg('--packets', 1000000)}_sub{arg('--substeps', 5)}"  # bench.py defaults
    rec = {"bytes_per_launch": corr, "bytes_per_launch_raw": raw, "fetch_kib": f_kib, "write_kib": w_kib,
           "dispatches": len(fetch), "note": "median dispatch; FETCH_SIZE doubled (gfx950 half-count)"}
    path = os.path.join(d, "traffic.json")  # copied into profiles/traffic.json once reviewed
    db = json.load(open(path)) if os.path.exists(path) else {}
    db[key] = rec
    json.dump(db, open(path, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(rec))


if __name__ == "__main__":
    main()
