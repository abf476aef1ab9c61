#!/bin/bash
# Round-5 session s: the CFL read-back copy on its own stream (off the QG
# stream's chain).  QG/driver tests, then driver-step A/B at 1.25e5 and 1e6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_qg.py tests/test_gpu_ode23.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
A="--no-cpu-baseline --no-fma --no-forecast --ode23-steps 0 --steps 20 --driver-steps 100"
timeout -k 10 500 bash tools/gpu_ab.sh r5s/125k new=default head=build/var/head.so -- $A --packets 125000 &&
timeout -k 10 500 bash tools/gpu_ab.sh r5s/1m new=default head=build/var/head.so -- $A --packets 1000000
