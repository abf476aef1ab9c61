#!/bin/bash
# Round 4: hazard checker + adversarial overlap tests, the stream tests, smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hazard.py tests/test_gpu_parity.py -k "hazard or streams or adversarial or single_launch or checker or bench_configuration" -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -15 $OUT/pytest.log
