#!/bin/bash
# Secondary rows: spectral + xka GPU tests, the config-5 study and the rows
# bench with their kernels' VALU fractions (tools/pmc_rows.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_rsw.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_rows.log 2>&1; rc=$?
tail -3 $OUT/pytest_rows.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_spectral.py --packets 1048576 --steps 1 > $OUT/spectral.json 2>&1 || exit $?
timeout -k 10 300 python tools/bench_rows.py > $OUT/rows.json 2>&1 || exit $?
bash tools/pmc_rows.sh $OUT/pmcrows
