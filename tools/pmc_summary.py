"""Per-kernel summary of tools/pmc_any.sh's passes: for every kernel name the
median over its dispatches of each counter and of the dispatch duration, and
the derived figures of MI355X_MICROARCH.md's PMC recipe:
  valu_issue   = SQ_INSTS_VALU x 64 / duration / 39.32e12 (fp64 lane-op peak at 2.4 GHz)
  lds_conflict = SQ_LDS_IDX_ACTIVE / (SQ_LDS_IDX_ACTIVE - SQ_LDS_BANK_CONFLICT)
  wait_frac    = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  hbm_gbs      = (2 x FETCH_SIZE + WRITE_SIZE) KiB / duration (gfx950 FETCH_SIZE counts half)
usage: python tools/pmc_summary.py <outdir>"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    return re.sub(r"\(.*", "", name).replace("void ", "").replace("swrt::", "")[:60]


def main(out):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for path in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {}
    for k, cs in vals.items():
        med = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}
        d = sorted(durs[k])[len(durs[k]) // 2] * 1e-9
        rec = {"dispatches": len(cs.get("SQ_WAVES", [])), "us": round(d * 1e6, 2)}
        rec.update({c: v for c, v in med.items()})
        if "SQ_INSTS_VALU" in med and d > 0:
            rec["valu_issue"] = med["SQ_INSTS_VALU"] * 64 / d / 39.3216e12
        if med.get("SQ_LDS_IDX_ACTIVE", 0) > med.get("SQ_LDS_BANK_CONFLICT", 0):
            rec["lds_conflict"] = med["SQ_LDS_IDX_ACTIVE"] / (med["SQ_LDS_IDX_ACTIVE"] - med["SQ_LDS_BANK_CONFLICT"])
        if med.get("SQ_WAVE_CYCLES"):
            rec["wait_frac"] = med.get("SQ_WAIT_ANY", 0) / med["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med and d > 0:
            rec["hbm_mb"] = (2 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024 / 1e6
            rec["hbm_gbs"] = rec["hbm_mb"] * 1e6 / d / 1e9
        res[k] = rec
    json.dump(res, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
