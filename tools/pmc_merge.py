"""Merge the rocprofv3 --pmc passes of tools/pmc_collect.sh into one record
per bench configuration: median over the dispatches of the packet kernel
(tile_leapfrog_kernel) of every counter, and the median dispatch duration of
those passes.  Writes <outdir>/pmc.json; `--install` merges it into
profiles/pmc.json, which bench.py reads for its roofline.

Units (MI355X_MICROARCH.md §HBM / §LDS / SQ PMC rows): FETCH_SIZE and
WRITE_SIZE in KiB, FETCH_SIZE counting half the bytes of wide streaming
reads on gfx950 (bench.py doubles it); SQ_* summed over the chip;
SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES and SQ_WAIT_ANY in quad-cycles;
SQ_LDS_IDX_ACTIVE / SQ_LDS_BANK_CONFLICT in LDS-array cycles.
usage: python tools/pmc_merge.py <outdir> [bench args...] | --install <outdir/pmc.json>"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PMC_KERNEL: a substring of the kernel name to merge (default: the bench's packet kernel)
KERNEL = os.environ.get("PMC_KERNEL", "tile_leapfrog_kernel")


def config_key(args):
    def arg(name, default):
        return args[args.index(name) + 1] if name in args else default
    key = f"{arg('--mode', 'blend')}_nx{arg('--nx', '512')}_N{arg('--packets', '1000000')}_sub{arg('--substeps', '5')}"
    iv = int(arg("--intervals", "1"))
    return key + (f"_iv{iv}" if iv > 1 else "") + ("_fma" if arg("--gather-mode", "0") == "1" else "")


def main():
    if sys.argv[1] == "--install":
        rec = json.load(open(sys.argv[2]))
        path = os.path.join(ROOT, "profiles", "pmc.json")
        db = json.load(open(path)) if os.path.exists(path) else {}
        db.update(rec)
        json.dump(db, open(path, "w"), indent=1, sort_keys=True)
        print("installed", list(rec))
        return
    d, args = sys.argv[1], sys.argv[2:]
    vals = collections.defaultdict(list)
    durs, name = [], ""
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r.get("Kernel_Name", ""):
                continue
            name = r["Kernel_Name"]
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if not vals:
        sys.exit("no packet-kernel rows")
    rec = {"kernel": name, "dispatches": len(vals.get("SQ_INSTS_VALU", [])),
           "pmc_kernel_ns": sorted(durs)[len(durs) // 2]}
    for c, v in vals.items():
        v.sort()
        rec[c] = v[len(v) // 2]
    rec["source"] = "rocprofv3 --pmc passes (tools/pmc_collect.sh), median dispatch"
    # bind the counters to the device code they were collected on (bench.py
    # refuses a record whose hash differs from the library it times)
    sys.path.insert(0, ROOT)
    from swraytracing_amd._lib import device_code_sha256
    rec["code_object_sha256"] = device_code_sha256()
    key = config_key(args)
    if KERNEL != "tile_leapfrog_kernel":
        key = re.sub(r"\W+", "_", KERNEL).strip("_") + "__" + key
    out = {key: rec}
    json.dump(out, open(os.path.join(d, "pmc.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
