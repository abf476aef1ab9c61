#!/bin/bash
# GPU-box session: `bash tools/gpu_run.sh <step>...` with steps
#   test   smoke + the GPU parity suite
#   bench  the default bench.py line (what the driver runs)
#   prof   the metric phase under rocprofv3 --kernel-trace --stats
#   phase  per-workgroup phase stamps (build/var/phase*.so) at 1e6 and 1.25e5
#   ab     bench A/B of build/var/*.so variants (AB_VARIANTS, AB_ARGS)
# Each GPU step has its own time limit; a crash/timeout (rc >= 124) ends the
# session immediately (no further GPU work), ordinary test failures do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${SESSION:-s}
mkdir -p "$OUT"
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
for s in "$@"; do
  case $s in
    test)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    bench)
      step bench 600 python bench.py ;;
    prof)
      export TMPDIR=/tmp
      step prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
        python3 "$ROOT/bench.py" --no-cpu-baseline --driver-steps 0 --ode23-steps 0 --no-fma --no-forecast ;;
    phase)
      for v in ${PHASE_LIBS:-phase}; do
        for n in 1000000 125000; do
          SWRT_LIB_PATH=build/var/$v.so step phase_${v}_$n 300 python tools/phase_timing.py --packets $n \
            --dump "$OUT/phase_${v}_$n.npz"
        done
      done ;;
    ab)
      step ab 1000 bash tools/gpu_ab.sh "${SESSION:-s}/ab" $AB_VARIANTS -- $AB_ARGS ;;
  esac
done
exit 0
