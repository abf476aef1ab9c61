#!/bin/bash
# Round 4: QG first-pass planes per workgroup beside packets (A/B in one box) + the new tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_qg.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_qg.log 2>&1 || { tail -30 $OUT/pytest_qg.log; exit 1; }
tail -1 $OUT/pytest_qg.log
for i in 1 2; do
for rv in 4 2 1; do
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-fma --ode23-steps 0 --forecast-intervals 1 --qg-rows-vecs $rv > $OUT/rv${rv}_$i.json 2> $OUT/rv${rv}_$i.err || { tail -20 $OUT/rv${rv}_$i.err; exit 1; }
echo "rows_vecs=$rv run $i"; python tools/summarize_bench.py $OUT/rv${rv}_$i.json | grep driver
done
done
