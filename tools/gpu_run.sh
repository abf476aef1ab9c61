#!/bin/bash
# GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash/timeout (rc >= 124) ends the
# session immediately (no further GPU work), ordinary test failures do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "FATAL: $name rc=$rc, stopping"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 400 python bench.py
  export TMPDIR=/tmp
  step prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --driver-steps 0 --ode23-steps 0 --no-fma --no-forecast
fi
exit 0
