#!/bin/bash
# GPU tests; then driver-step A/B: tile-workgroup size and packet streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3i
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/session_r3h.sh
timeout -k 10 120 python tools/bench_pipeline.py > $OUT/pipeline.json 2> $OUT/pipeline.err || exit $?
python -c "import json; d=json.load(open('$OUT/pipeline.json')); print('pipeline step_ms %.4f packets_ms %.4f pde %.4f'%(d['step_ms'], d['packets_ms'], d['pde_ms']))"
