#!/bin/bash
# experiment session: parity of the packet kernels, A/B bench sweep, phase stamps
# usage: tools/session_exp.sh "<sweep spec>" ... (sweep.sh syntax: [lib.so::]bench flags)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_exp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep.sh "$@" || exit $?
if [ -f build/variants/phase.so ]; then
  SWRT_LIB_PATH=build/variants/phase.so timeout -k 10 200 python tools/phase_timing.py --samples 12 --dump gpurun_out/phase_raw_exp.npz > gpurun_out/phase_exp.log 2>&1; echo phase rc=$?
fi
if [ -n "$PMC_GROUP" ]; then
  bash tools/pmc_counters.sh "--steps 10 --warmup 2 --no-cpu-baseline" "$PMC_GROUP" > gpurun_out/pmc_exp.log 2>&1; echo pmc rc=$?
fi
