#!/bin/bash
# Round-5 session k: ode23 event waits by polling vs hipEventSynchronize.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 12 --steps 5"
timeout -k 10 600 bash tools/gpu_ab.sh r5k/ab sync=default spin=build/var/spin.so -- $B
