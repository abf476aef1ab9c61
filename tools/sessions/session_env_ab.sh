#!/bin/bash
# driver-pipeline A/B over the values of one environment switch, alternating:
#   VAR=SWRT_X VALUES="0 1" bash tools/session_env_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
i=0
for rep in 1 2; do
  for v in $VALUES; do
    i=$((i+1))
    env "$VAR=$v" timeout -k 10 200 python tools/bench_pipeline.py $PIPE_ARGS > $OUT/envab_$i.json 2>&1 || exit $?
    echo "$VAR=$v $(tail -1 $OUT/envab_$i.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pde %.4f cfl %.4f snap %.4f pk %.4f step %.4f" % (d["pde_ms"], d["cfl_ms"], d["snapshot_ms"], d["packets_ms"], d["step_ms"]))')"
  done
done
