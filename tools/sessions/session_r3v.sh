#!/bin/bash
# Driver step: snapshot-before-speed queue order vs the old order, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3v
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 10 --driver-steps 40"
for i in 1 2 3; do
  for v in old new; do
    F=""; [ $v = old ] && F="--old-order"
    timeout -k 10 200 python tools/ab_driver_order.py $F $B > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python -c "
import json
d=json.loads([l for l in open('$OUT/bench_${v}_$i.json') if l.startswith('{')][0])
print('$v $i driver %.4f ms  headline %.3e' % (d['driver_step']['ms_per_pde_step'], d['value']))"
  done
done
