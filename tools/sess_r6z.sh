#!/bin/bash
# Round-6 final validation after the ode23 launch change: PMC of the packet
# kernel on this device code (1e6 and 1.25e5, installed into profiles/pmc.json
# on the box so the bench's roofline binds to it), then the default bench
# line, the rocprofv3 stats of the metric phase, smoke and the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=${SESSION:-r6z}
O=gpurun_out/$S
mkdir -p $O
export TMPDIR=/tmp
B="--steps 12 --warmup 2 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --packet-streams 1"
timeout -k 10 420 bash tools/pmc_collect.sh $O/m1 "$B" || exit $?
timeout -k 10 420 bash tools/pmc_collect.sh $O/m125 "$B --packets 125000" || exit $?
python3 tools/pmc_merge.py --install $O/m1/pmc.json && python3 tools/pmc_merge.py --install $O/m125/pmc.json || exit 1
cp profiles/pmc.json $O/pmc_installed.json
SESSION=$S bash tools/sess_r6.sh bench prof test
