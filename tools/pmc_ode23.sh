#!/bin/bash
# PMC counters of the drivers' ode23 attempt kernel (tile_ode23_kernel<0>:
# stages 2-4 of a Bogacki-Shampine attempt fused): bench.py's driver_step_ode23
# under one rocprofv3 --pmc pass per counter group (kernel trace only beside
# --pmc), merged by tools/pmc_merge.py with PMC_KERNEL -> <outdir>/pmc.json.
# usage: tools/pmc_ode23.sh <outdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$1
BARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 2 --driver-warmup 2 --driver-warm-s 0 --packet-streams 1"
mkdir -p "$OUT"
export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES"
         "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE")
i=0
for g in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$ROOT/bench.py" $BARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($g) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
PMC_KERNEL="tile_ode23_kernel<0" python3 tools/pmc_merge.py "$OUT" $BARGS
