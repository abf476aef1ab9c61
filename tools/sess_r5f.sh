#!/bin/bash
# Round-5 session f: ode23 attempts split over the two packet streams, maxima
# read from host-mapped memory, ramp-up guesses; the PDE step queued before
# the ode23 interval.  Tests, A/B against the previous library, a trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5f
mkdir -p $O/ode23
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ode23.py tests/test_gpu_qg.py -x -v --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
B="--no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 8 --steps 5"
timeout -k 10 500 bash tools/gpu_ab.sh r5f/ab new=default prev=build/var/prev.so -- $B &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ode23 -o ode23 --output-format csv -- \
  python3 bench.py $B > $O/ode23/bench.json 2> $O/ode23/bench.err
