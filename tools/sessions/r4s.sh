#!/bin/bash
# Round 4: driver step with the PDE serialized on the packet stream (alone-optimal
# kernel shapes, speculative steps) against the separate QG stream; in-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4s
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
for cfg in "1 1" "0 1" "0 0"; do
set -- $cfg
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-fma --ode23-steps 0 --forecast-intervals 1 --qg-stream $1 --qg-update-cols $2 > $OUT/s$1u$2_$i.json 2> $OUT/s$1u$2_$i.err || { tail -20 $OUT/s$1u$2_$i.err; exit 1; }
echo "qg_stream=$1 update_cols=$2 run $i"; python tools/summarize_bench.py $OUT/s$1u$2_$i.json | grep -i "driver\|pde"
done
done
