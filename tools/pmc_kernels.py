"""Per-kernel VALU-issue fraction from the rocprofv3 --pmc runs of
tools/pmc_rows.sh: for every kernel name, its longest dispatch (the timed call, not the
warm-ups): SQ_INSTS_VALU (wave-instructions, chip total), the dispatch
duration (counter-collection Start/End timestamps), the measured engine clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration) and
  valu_frac = SQ_INSTS_VALU x 64 lanes / duration / (256 CUs x 4 SIMDs x 16 lanes x 2.4 GHz)
(one fp64 or unpacked fp32 VALU op per lane per lane-slot; a packed fp32 op
counts once, so the fp32 packed kernel's FLOP rate is up to 2x this).
usage: python tools/pmc_kernels.py <outdir>  (reads <outdir>/*/run_counter_collection.csv)"""
import collections
import csv
import glob
import json
import os
import sys

PEAK = 256 * 4 * 16 * 2.4e9
KEEP = ("xka_", "spectral_", "omega_hist", "tile_leapfrog", "ode23")


def main(out):
    rec = collections.defaultdict(lambda: collections.defaultdict(dict))
    for path in glob.glob(os.path.join(out, "*", "run_counter_collection.csv")):
        src = os.path.basename(os.path.dirname(path))
        for row in csv.DictReader(open(path)):
            name = row["Kernel_Name"]
            if not any(k in name for k in KEEP):
                continue
            d = rec[(src, name)][row["Dispatch_Id"]]
            d[row["Counter_Name"]] = float(row["Counter_Value"])
            d["ns"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    res = {}
    for (src, name), disp in sorted(rec.items()):
        rows = [d for d in disp.values() if "SQ_INSTS_VALU" in d and d["ns"] > 0]
        if not rows:
            continue
        top = max(rows, key=lambda d: d["ns"])
        med = {k: top.get(k, 0.0) for k in ("SQ_INSTS_VALU", "SQ_WAVES", "ns")}
        s = med["ns"] * 1e-9
        r = {"source": src, "dispatches": len(rows), "valu_per_dispatch": med["SQ_INSTS_VALU"],
             "waves": med["SQ_WAVES"], "ms": s * 1e3, "valu_frac": med["SQ_INSTS_VALU"] * 64 / s / PEAK}
        if "GRBM_GUI_ACTIVE" in top:
            clk = top["GRBM_GUI_ACTIVE"] / 8 / s
            r["clock_ghz_measured"] = clk / 1e9
            r["valu_frac_at_measured_clock"] = r["valu_frac"] * 2.4e9 / clk
        res[name] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
