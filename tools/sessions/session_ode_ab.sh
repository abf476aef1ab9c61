#!/bin/bash
# ode23 interval A/B: tools/bench_pipeline.py --ode23 per build (SWRT_LIB_PATH), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
i=0
for rep in 1 2; do
  for lib in "$@"; do
    i=$((i+1))
    SWRT_LIB_PATH=$lib timeout -k 10 200 python tools/bench_pipeline.py --ode23 --steps 4 > $OUT/ode_$i.json 2>&1 || exit $?
    echo "$lib $(tail -1 $OUT/ode_$i.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); o=d["ode23"]; print("ode23 interval %.3f ms, %d rhs, %.1f us/rhs" % (o["interval_ms"], o["rhs_evals"], o["ms_per_rhs_eval"]*1e3))')"
  done
done
