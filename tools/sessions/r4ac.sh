#!/bin/bash
# Round 4: re-binning interval (15/20/25/30 steps) and packet streams (2/4) at
# 1e6 on the final tree; in-box A/B of the metric only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4ac
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
for cfg in "20 2" "15 2" "25 2" "30 2" "20 4"; do
set -- $cfg
timeout -k 10 200 python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --rebin-every $1 --packet-streams $2 > $OUT/r$1s$2_$i.json 2> $OUT/r$1s$2_$i.err || { tail -20 $OUT/r$1s$2_$i.err; exit 1; }
echo "rebin=$1 streams=$2 run $i $(python tools/summarize_bench.py $OUT/r$1s$2_$i.json | head -1)"
done
done
