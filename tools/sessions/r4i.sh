#!/bin/bash
# Round 4: speculative PDE steps A/B (driver step at 1e6 and the forecast's shard sizes, 100 steps each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4i
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
for sp in 0 1; do
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-fma --ode23-steps 0 --forecast-intervals 1 --speculate $sp > $OUT/spec${sp}_$i.json 2> $OUT/spec${sp}_$i.err || { tail -20 $OUT/spec${sp}_$i.err; exit 1; }
echo "speculate=$sp run $i"; python tools/summarize_bench.py $OUT/spec${sp}_$i.json | grep driver
done
done
