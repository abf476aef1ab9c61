#!/bin/bash
# Final code, part A: smoke, GPU suite, tile-kernel PMC (bit-exact + FMA).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3fa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/pmc_collect.sh $OUT/pmc || exit $?
bash tools/pmc_collect.sh $OUT/pmc_fma "--steps 12 --warmup 2 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --packet-streams 1 --gather-mode 1" || exit $?
