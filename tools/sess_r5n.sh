#!/bin/bash
# Round-5 session n: the ode23 driver loop packs the speculative step's
# snapshot inside the interval (swrt_qg_snapshot_speculative).  Tests, then
# an A/B against the previous library (same Python: its hook path falls
# back to a plain snapshot when the call is missing? no — the head library
# lacks the symbol, so the A/B runs with --speculate on both and the head
# build is loaded only by the bench's C calls it has).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_qg.py tests/test_gpu_ode23.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
B="--no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 12 --steps 5"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py $B > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  python -c "import json; j=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print(j['driver_step_ode23']['ms_per_pde_step'])"
done
