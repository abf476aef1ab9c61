#!/bin/bash
# Next-bin keys led by half a cycle of group-velocity drift: parity tests, then A/B vs the previous build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3aj
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_intervals.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 80"
for i in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then export SWRT_LIB_PATH=$PWD/build_ab/libswrt_head.so; else unset SWRT_LIB_PATH; fi
    timeout -k 10 200 python bench.py $B > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { tail -5 $OUT/bench_${v}_$i.err; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('$OUT/bench_${v}_$i.json') if l.startswith('{')][0])
print('$v $i %.4e ms/step %.4f driver %.4f' % (d['value'], d['ms_per_step'], d['driver_step']['ms_per_pde_step']))"
  done
done
unset SWRT_LIB_PATH
for n in 125000 250000; do
  for v in head new; do
    if [ $v = head ]; then export SWRT_LIB_PATH=$PWD/build_ab/libswrt_head.so; else unset SWRT_LIB_PATH; fi
    timeout -k 10 200 python bench.py $B --driver-steps 0 --packets $n > $OUT/n${n}_${v}.json 2> $OUT/n${n}_${v}.err || exit 1
    python -c "
import json
d=json.loads([l for l in open('$OUT/n${n}_${v}.json') if l.startswith('{')][0])
print('n $n $v %.4e' % d['value'])"
  done
done
