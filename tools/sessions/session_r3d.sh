#!/bin/bash
# Small-shard diagnosis: which fixed cost or density effect bounds a
# 1.25e5-packet launch.  Timing variants + issue/wait PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r3d
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --steps 40 --warmup 5"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 120 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0]); print('$name', '%.3e'%d['value'], 'launch_ms', d['roofline']['avg_launch_ms'], 'steps/launch', d['config']['steps_per_launch'])"
}
run base_1e6
run base_125k --packets 125000 --tile-cells 16
run strat_125k --packets 125000 --tile-cells 16 --positions stratified
run sub20_125k --packets 125000 --tile-cells 16 --substeps 20 --rebin-every 20
run sub20_1e6 --substeps 20 --rebin-every 20
run nx256_125k --packets 125000 --nx 256 --tile-cells 16
run nx256_1e6 --packets 1000000 --nx 256 --tile-cells 16
run cs1_125k --packets 125000 --tile-cells 16 --cell-sort 1
run lead0_125k --packets 125000 --tile-cells 16 --rebin-every 5
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
G="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
for cfg in "125000 16" "125000 32" "1000000 16"; do
  set -- $cfg
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$OUT/pmc_N$1_t$2" -o run \
    -- python3 "$ROOT/bench.py" $B --steps 12 --warmup 2 --packets $1 --tile-cells $2 > "$OUT/pmc_N$1_t$2.log" 2>&1 || exit $?
  echo "pmc N=$1 tile=$2 done"
done
