#!/bin/bash
# A/B on one box: one vs two packet streams, alternating, with the
# end-to-end driver step (longer warm-up).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3g
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 40 --ode23-steps 0"
for i in 1 2 3; do
  for ps in 1 2; do
    timeout -k 10 200 python bench.py --packet-streams $ps $B > $OUT/bench_ps${ps}_$i.json 2> $OUT/bench_ps${ps}_$i.err || exit $?
    python -c "import json; d=json.loads([l for l in open('$OUT/bench_ps${ps}_$i.json') if l.startswith('{')][0]); print('ps=$ps run $i', '%.4e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'launch %.4f'%d['roofline']['avg_launch_ms'], 'driver %.4f'%d['driver_step']['ms_per_pde_step'])"
  done
done
