#!/bin/bash
# Round-3 session: GPU tests (paired lanes, stored tracing, FMA mode), then
# the small-shard forecast with auto / one-lane launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ge 124 ]; then exit $rc; fi
for lanes in 0 1; do
  timeout -k 10 300 python bench.py --lanes-per-packet $lanes --no-cpu-baseline --driver-steps 0 --ode23-steps 0 \
    --no-fma > $OUT/bench_lanes$lanes.json 2> $OUT/bench_lanes$lanes.err || exit $?
  echo "bench lanes=$lanes done"
done
