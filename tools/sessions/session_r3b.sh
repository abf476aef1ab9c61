#!/bin/bash
# Small-shard diagnosis: per-workgroup phase stamps (diagnostic build) and
# PMC of the tile kernel at 1.25e5 packets, one and two lanes per packet.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r3b
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "125000 1" "125000 2" "1000000 1"; do
  set -- $cfg
  SWRT_LIB_PATH=$ROOT/build/variants/phase.so timeout -k 10 120 python tools/phase_timing.py --packets $1 \
    --lanes-per-packet $2 --samples 4 > $OUT/phase_N$1_l$2.json 2> $OUT/phase_N$1_l$2.err || exit $?
  echo "phase N=$1 lanes=$2 done"
done
BARGS="--packets 125000 --steps 12 --warmup 2 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0"
for lanes in 1 2; do
  i=0
  for g in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES" "SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$OUT/pmc_l$lanes/p$i" -o run \
      -- python3 "$ROOT/bench.py" $BARGS --lanes-per-packet $lanes > "$OUT/pmc_l${lanes}_p$i.log" 2>&1 || exit $?
    echo "pmc lanes=$lanes pass $i done"
  done
done
