#!/bin/bash
# A/B session: GPU parity tests on the in-tree build, then bench variants
# (alternating builds from build/ab/), each step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TESTS=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep.sh "$@"
