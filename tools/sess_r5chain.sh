#!/bin/bash
# Round-5 session: ode23 stage 1 chained to the previous interval
# (swrt_ode23_chain_next).  Tests, then the drivers' ode23 interval with the
# chain off / on (SWRT_ODE23_CHAIN), alternating, then a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5chain
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ode23.py tests/test_gpu_qg.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
A="--steps 1 --warmup 0 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps ${ODE23_STEPS:-13}"
for i in 1 2 3; do
  for ch in 0 1; do
    SWRT_ODE23_CHAIN=$ch timeout -k 10 200 python bench.py $A > $O/chain${ch}_$i.json 2> $O/chain${ch}_$i.err || exit $?
    python - $O/chain${ch}_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d.get("driver_step_ode23", {})
print(sys.argv[1], {k: o.get(k) for k in ("ms_per_pde_step", "ode23_per_interval", "clock_ghz_observed")})
PY
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py $A \
  > $O/trace_bench.log 2>&1 || exit $?
python tools/ode23_timeline.py $(python -c "import glob; print(sorted(glob.glob('$O/tr/**/*kernel_trace.csv', recursive=True))[0])") \
  --json $O/timeline.json > $O/timeline.txt && tail -16 $O/timeline.txt
