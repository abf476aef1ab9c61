#!/bin/bash
# Round-5 PMC session on the current device code: the bench's packet kernel
# at 1e6 and at the 8-GPU shard (1.25e5), then the QG PDE kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5pmc
mkdir -p $O
B="--steps 12 --warmup 2 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --packet-streams 1"
timeout -k 10 420 bash tools/pmc_collect.sh $O/m1 "$B" || exit $?
timeout -k 10 420 bash tools/pmc_collect.sh $O/m125 "$B --packets 125000" || exit $?
timeout -k 10 300 bash tools/pmc_qg.sh $O/qg || exit $?
ls $O/*/pmc.json $O/qg/qg_pmc.json
