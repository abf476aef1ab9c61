#!/bin/bash
# Round 4: J's last forward pass fused into the AB3 update — QG tests, then an
# in-box A/B of the driver step, the PDE alone and the shard forecast.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_qg.py -k 'update_column or speculative or fused or configs' -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_qg.log 2>&1 || { tail -30 $OUT/pytest_qg.log; exit 1; }
tail -1 $OUT/pytest_qg.log
for i in 1 2; do
for u in 1 0; do
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-fma --ode23-steps 0 --forecast-intervals 1 --qg-update-cols $u > $OUT/u${u}_$i.json 2> $OUT/u${u}_$i.err || { tail -20 $OUT/u${u}_$i.err; exit 1; }
echo "update_cols=$u run $i"; python tools/summarize_bench.py $OUT/u${u}_$i.json | grep -i "driver\|pde"
done
done
