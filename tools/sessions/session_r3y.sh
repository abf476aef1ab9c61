#!/bin/bash
# FFT vectors per workgroup (SWRT_FFT_GROUP 4 / 2 / 1): QG-only and driver step, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3y
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 20 --driver-steps 40"
run() {
  local name=$1 lib=$2
  if [ $lib = default ]; then unset SWRT_LIB_PATH; else export SWRT_LIB_PATH=$PWD/build_ab/libswrt_$lib.so; fi
  timeout -k 10 60 python tools/bench_qg.py > $OUT/qg_$name.json 2>/dev/null || exit $?
  timeout -k 10 200 python bench.py $B > $OUT/bench_$name.json 2> $OUT/bench_$name.err || exit $?
  python -c "
import json
q=json.loads([l for l in open('$OUT/qg_$name.json') if l.startswith('{')][0])
d=json.loads([l for l in open('$OUT/bench_$name.json') if l.startswith('{')][0])
print('$name qg %.4f ms  driver %.4f ms  headline %.3e' % (q['ms_per_step'], d['driver_step']['ms_per_pde_step'], d['value']))"
}
for i in 1 2 3; do
  run g4_$i default
  run g2_$i g2
  run g1_$i g1
done
