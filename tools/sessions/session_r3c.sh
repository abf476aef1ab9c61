#!/bin/bash
# GPU tests, then the forecast with 32-cell tiles (auto) vs 16-cell tiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cells in 0 16; do
  timeout -k 10 300 python bench.py --tile-cells $cells --no-cpu-baseline --driver-steps 0 --ode23-steps 0 \
    --no-fma > $OUT/bench_cells$cells.json 2> $OUT/bench_cells$cells.err || exit $?
  echo "bench cells=$cells done"
done
