#!/bin/bash
# PMC counters of every kernel a command runs: one rocprofv3 pass per counter
# group (kernel trace only beside --pmc; FETCH_SIZE and WRITE_SIZE in passes
# of their own), then tools/pmc_summary.py -> <outdir>/summary.json.
# usage: tools/pmc_any.sh <outdir> <python script> [args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES"
         "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE")
i=0
for g in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($g) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json"
