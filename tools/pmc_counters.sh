#!/bin/bash
# Collect PMC counters (one rocprofv3 pass per group) for the bench's hot kernel.
# usage: tools/pmc_counters.sh "<bench args>" "C1 C2 ..." ["C3 C4" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcc
mkdir -p "$OUT"
export TMPDIR=/tmp
BARGS=$1; shift
g=0
for group in "$@"; do
  g=$((g+1))
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-trace --output-format csv -d "$OUT/g$g" -o run -- python3 "$ROOT/bench.py" $BARGS > "$OUT/g$g.log" 2>&1
  rc=$?; echo "group $g ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$g.log"; [ $rc -ge 124 ] && exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "leapfrog" in r.get("Kernel_Name", ""):
            vals[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    v.sort()
    print(f"{k:60s} {c:28s} median {v[len(v)//2]:.4g}  n={len(v)}")
PY
