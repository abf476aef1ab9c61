#!/bin/bash
# Round-5 session p: SIMD-balanced busy waves in the 256-thread sparse shape
# (per-CU tickets).  Parity tests, then A/B against the previous library at
# the 8-GPU shard (1.25e5) and 2.5e5, and at 1e6 (must be unchanged).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_intervals.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
A="--no-cpu-baseline --no-fma --no-forecast --ode23-steps 0 --steps 40"
timeout -k 10 500 bash tools/gpu_ab.sh r5p/125k new=default head=build/var/head.so -- $A --packets 125000 &&
timeout -k 10 300 bash tools/gpu_ab.sh r5p/1m new=default head=build/var/head.so -- $A --packets 1000000 --driver-steps 0
