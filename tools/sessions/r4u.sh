#!/bin/bash
# Round 4: sparse-tile shape (256-thread workgroups) vs dense beside the PDE —
# the end-to-end driver forecast at the shard sizes; in-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4u
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
for sp in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-fma --ode23-steps 0 --forecast-intervals 1 --sparse-tiles $sp > $OUT/sp${sp}_$i.json 2> $OUT/sp${sp}_$i.err || { tail -20 $OUT/sp${sp}_$i.err; exit 1; }
echo "sparse=$sp run $i"; python tools/summarize_bench.py $OUT/sp${sp}_$i.json | grep -v ode23
done
done
