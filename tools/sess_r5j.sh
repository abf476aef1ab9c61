#!/bin/bash
# Round-5 session j: ode23 re-binning cadence A/B (every 1 / 2 / 4 calls).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5j
mkdir -p $O
SWRT_LIB_PATH=build/var/orb4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ode23.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest_orb4.log 2>&1 || exit $?
B="--no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 12 --steps 5"
timeout -k 10 700 bash tools/gpu_ab.sh r5j/ab r1=default r2=build/var/orb2.so r4=build/var/orb4.so -- $B
