#!/bin/bash
# driver-pipeline A/B: tools/bench_pipeline.py per build (SWRT_LIB_PATH), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
i=0
for rep in 1 2; do
  for lib in "$@"; do
    i=$((i+1))
    SWRT_LIB_PATH=$lib timeout -k 10 200 python tools/bench_pipeline.py > $OUT/pipe_$i.json 2>&1 || exit $?
    echo "$lib $(tail -1 $OUT/pipe_$i.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pde %.4f cfl %.4f snap %.4f pk %.4f step %.4f" % (d["pde_ms"], d["cfl_ms"], d["snapshot_ms"], d["packets_ms"], d["step_ms"]))')"
  done
done
