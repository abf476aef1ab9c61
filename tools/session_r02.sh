#!/bin/bash
# Round-2 GPU session: smoke, GPU parity suite, bench A/B of the launch
# order (longest-first vs spatial tile order), rocprofv3 kernel stats.
# Each GPU step has its own time limit; rc >= 124 (timeout/abort/crash) ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "FATAL: $name rc=$rc"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = ab ]; then
  shift
  bash tools/sweep.sh "$@" || exit $?
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --steps 50
  step bench 400 python bench.py
fi
exit 0
