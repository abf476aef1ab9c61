#!/bin/bash
# Round-6 GPU session: `SESSION=<name> bash tools/sess_r6.sh <step>...`
#   new    the GPU tests this round added or changed (ode23 at scale, hook
#          refusal, chain rewrite, lost packets, sharded drivers)
#   test   smoke + the whole GPU suite (no -x: every failure reported)
#   bench  the default bench.py line (what the driver runs)
#   prof   the metric phase under rocprofv3 --kernel-trace --stats
# Each GPU step has its own time limit; a crash or timeout (rc >= 124) ends
# the session (no further GPU work); ordinary test failures do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${SESSION:-r6}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -3 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "FATAL: $name rc=$rc, stopping"; exit $rc; fi
  return 0
}
NEW="tests/test_gpu_ode23.py tests/test_gpu_hazard.py tests/test_dist_gpu.py"
for s in "$@"; do
  case $s in
    new)
      step pytest_new 900 python -u -m pytest $NEW -m gpu -v --timeout 300 --timeout-method thread ;;
    test)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    bench)
      step bench 700 python bench.py
      cp "$OUT/bench.log" "$OUT/bench_full.log"
      grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true ;;
    prof)
      step prof 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
        python3 bench.py --no-cpu-baseline --driver-steps 0 --ode23-steps 0 --no-fma --no-forecast ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
