#!/bin/bash
# HBM bytes of the QG PDE kernels (tools/bench_qg.py, no packets): FETCH_SIZE
# and WRITE_SIZE in passes of their own with the kernel trace, then
# tools/pmc_qg_summary.py -> <outdir>/qg_pmc.json.
# usage: tools/pmc_qg.sh <outdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for g in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$OUT/q$i" -o run \
    -- python3 "$ROOT/tools/bench_qg.py" > "$OUT/q$i.log" 2>&1 || { tail -5 "$OUT/q$i.log"; exit 1; }
  echo "qg pmc pass $i ($g) done"
done
python3 tools/pmc_qg_summary.py "$OUT" > "$OUT/qg_pmc.json"
