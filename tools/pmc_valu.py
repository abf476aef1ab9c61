"""Merge SQ counter passes (tools/pmc_counters.sh -> gpurun_out/pmcc/g*/)
into profiles/valu.json under the bench's config key: median over the
dispatches of the leapfrog tile kernel.  bench.py reads SQ_INSTS_VALU from it
for `valu_roofline`.  usage: python tools/pmc_valu.py <pmcc dir> <key> <kernel note>"""
import collections
import csv
import glob
import json
import os
import sys

NAMES = ["SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT",
         "SQ_WAVES", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"]


def main():
    d, key, note = sys.argv[1], sys.argv[2], sys.argv[3]
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "leapfrog" in r.get("Kernel_Name", ""):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    rec = {"kernel": note}
    for n in NAMES:
        if vals.get(n):
            v = sorted(vals[n])
            rec[n + ("_quad_cycles" if n == "SQ_ACTIVE_INST_VALU" else "")] = v[len(v) // 2]
    rec["note"] = ("median over the profiled dispatches (tools/pmc_counters.sh); SQ_* summed over the chip; "
                   "SQ_ACTIVE_INST_VALU/WAVE_CYCLES/WAIT_ANY in quad-cycles (MI355X_MICROARCH.md)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "profiles", "valu.json")
    db = json.load(open(path)) if os.path.exists(path) else {}
    db[key] = rec
    json.dump(db, open(path, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(rec))


if __name__ == "__main__":
    main()
