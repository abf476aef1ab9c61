#!/bin/bash
# PMC on the current code: the headline tile kernel (bit-exact and FMA
# configurations) and the QG PDE kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3k
mkdir -p $OUT
bash tools/pmc_collect.sh $OUT/pmc || exit $?
bash tools/pmc_collect.sh $OUT/pmc_fma "--steps 12 --warmup 2 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --packet-streams 1 --gather-mode 1" || exit $?
timeout -k 10 60 python tools/bench_qg.py > $OUT/qg_time.json 2>&1 || exit $?
cat $OUT/qg_time.json
bash tools/pmc_qg.sh $OUT/qg || exit $?
