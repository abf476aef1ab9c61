#!/bin/bash
# Round-5 session i: ode23 first attempt from the device's step size, the
# next QG step queued through the ode23 hook.  Tests, bench reps, a trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5i
mkdir -p $O/ode23
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
B="--no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 8 --steps 5"
for i in 1 2; do
  timeout -k 10 200 python bench.py $B > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  python -c "import json; j=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print(j['driver_step_ode23'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ode23 -o ode23 --output-format csv -- \
  python3 bench.py $B > $O/ode23/bench.json 2> $O/ode23/bench.err
