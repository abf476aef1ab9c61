#!/bin/bash
# Slot-use marking without the per-call join (driver): QG/driver tests, then
# driver-step A/B against HEAD's build on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3ai
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_qg.py tests/test_gpu_stored.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 20 --driver-steps 40"
for i in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then export SWRT_LIB_PATH=$PWD/build_ab/libswrt_head.so; else unset SWRT_LIB_PATH; fi
    timeout -k 10 200 python bench.py $B > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { tail -5 $OUT/bench_${v}_$i.err; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('$OUT/bench_${v}_$i.json') if l.startswith('{')][0])
print('$v $i driver %.4f ms  headline %.3e' % (d['driver_step']['ms_per_pde_step'], d['value']))"
  done
done
