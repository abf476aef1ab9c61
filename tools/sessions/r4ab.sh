#!/bin/bash
# Round 4: the PDE fusions forced beside packet launches (debug value 2) vs
# the default gating — driver step and the shard forecast (the 8-GPU shard
# now runs the sparse-tile shape); in-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4ab
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
for cfg in "1 1" "2 2" "1 2"; do
set -- $cfg
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-fma --ode23-steps 0 --forecast-intervals 1 --qg-jfuse $1 --qg-update-cols $2 > $OUT/j$1u$2_$i.json 2> $OUT/j$1u$2_$i.err || { tail -20 $OUT/j$1u$2_$i.err; exit 1; }
echo "jfuse=$1 update_cols=$2 run $i"; python tools/summarize_bench.py $OUT/j$1u$2_$i.json | grep -i "driver\|pde"
done
done
