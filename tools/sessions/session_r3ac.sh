#!/bin/bash
# Packet streams 2 / 4 with 4 (default) and 8 hardware queues per process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3ac
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --driver-steps 40"
for i in 1 2; do
  for q in 4 8; do
    for s in 2 4; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py $B --packet-streams $s > $OUT/bench_q${q}_s${s}_$i.json 2> $OUT/bench_q${q}_s${s}_$i.err || { tail -5 $OUT/bench_q${q}_s${s}_$i.err; exit 1; }
      python -c "
import json
d=json.loads([l for l in open('$OUT/bench_q${q}_s${s}_$i.json') if l.startswith('{')][0])
print('queues $q streams $s run $i: %.4e  ms/step %.4f driver %.4f' % (d['value'], d['ms_per_step'], d['driver_step']['ms_per_pde_step']))"
    done
  done
done
