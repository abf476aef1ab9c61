#!/bin/bash
# tail-split experiment: parity of the split launches, bench sweep, phase stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tile_kernel" --timeout 120 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_split.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep.sh "--tail-split 0" "--tail-split 8" "--tail-split 16" "--tail-split 32" "--tail-split 64" "--tail-split 0" "--tail-split 16" "--tail-split 32" || exit $?
SWRT_LIB_PATH=build/variants/phase.so timeout -k 10 200 python tools/phase_timing.py --samples 12 --tail-split 32 --dump gpurun_out/phase_raw32.npz > gpurun_out/phase32.log 2>&1; echo phase rc=$?
