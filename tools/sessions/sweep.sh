#!/bin/bash
# bench variants in one session (each with its own time limit; stop on crash).
# Each argument: "[lib.so::]bench flags"  (lib.so = alternative build via SWRT_LIB_PATH)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
i=0
while [ $# -gt 0 ]; do
  spec=$1; shift; i=$((i+1))
  lib=""; args=$spec
  if [[ "$spec" == *"::"* ]]; then lib=${spec%%::*}; args=${spec#*::}; fi
  SWRT_LIB_PATH=$lib timeout -k 10 240 python bench.py --no-cpu-baseline $args > $OUT/sweep_$i.log 2>&1
  rc=$?
  echo "[$rc] $spec :: $(grep '^{' $OUT/sweep_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g pkt-steps/s  launch %.1f us" % (d["value"], d["roofline"]["avg_launch_ms"]*1e3))' 2>/dev/null)"
  if [ $rc -ge 124 ]; then echo FATAL; exit $rc; fi
done
