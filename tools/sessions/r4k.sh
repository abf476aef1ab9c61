#!/bin/bash
# Round 4: in-box A/B of the QG column/Jacobian fusion and speculative steps (driver step + forecast).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4k
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
for cfg in "1 1" "0 1" "1 0" "0 0"; do
set -- $cfg
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-fma --ode23-steps 0 --forecast-intervals 1 --qg-jfuse $1 --speculate $2 > $OUT/j$1s$2_$i.json 2> $OUT/j$1s$2_$i.err || { tail -20 $OUT/j$1s$2_$i.err; exit 1; }
echo "jfuse=$1 speculate=$2 run $i"; python tools/summarize_bench.py $OUT/j$1s$2_$i.json | grep driver
done
done
