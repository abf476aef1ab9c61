#!/bin/bash
# Round 4: read-backs handed to the host by the kernels themselves (the QG
# Jacobian pass's CFL max, the ode23 attempt's error max) — QG/ode23 tests,
# then an in-box A/B of the driver steps and the shard forecast.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_qg.py tests/test_gpu_ode23.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_qg.log 2>&1 || { tail -30 $OUT/pytest_qg.log; exit 1; }
tail -1 $OUT/pytest_qg.log
for i in 1 2; do
for h in 1 0; do
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-fma --forecast-intervals 1 --qg-host-handoff $h --ode23-host-handoff $h > $OUT/h${h}_$i.json 2> $OUT/h${h}_$i.err || { tail -20 $OUT/h${h}_$i.err; exit 1; }
echo "handoff=$h run $i"; python tools/summarize_bench.py $OUT/h${h}_$i.json | grep -i "driver\|pde"
done
done
