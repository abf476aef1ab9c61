#!/bin/bash
# Driver step: speculative next PDE step vs the round trip, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3z
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_qg.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_qg.log 2>&1 || { tail -30 $OUT/pytest_qg.log; exit 1; }
tail -1 $OUT/pytest_qg.log
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 10 --driver-steps 40"
for i in 1 2 3; do
  for v in base spec; do
    F=""; [ $v = spec ] && F="--spec"
    timeout -k 10 200 python tools/ab_driver_spec.py $F $B > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { tail -5 $OUT/bench_${v}_$i.err; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('$OUT/bench_${v}_$i.json') if l.startswith('{')][0])
print('$v $i driver %.4f ms  headline %.3e' % (d['driver_step']['ms_per_pde_step'], d['value']))"
  done
done
