#!/bin/bash
# Packet workgroups of 448 lanes (a wave slot free on half the SIMDs for the
# QG stream) with one-vector FFT workgroups: parity subset, then driver A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3x
mkdir -p $OUT
export SWRT_LIB_PATH=$PWD/build_ab/libswrt_nt448.so
true
true
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 20 --driver-steps 40"
run() {
  local name=$1 lib=$2
  if [ $lib = default ]; then unset SWRT_LIB_PATH; else export SWRT_LIB_PATH=$PWD/build_ab/libswrt_$lib.so; fi
  timeout -k 10 200 python bench.py $B > $OUT/bench_$name.json 2> $OUT/bench_$name.err || exit $?
  python -c "
import json
d=json.loads([l for l in open('$OUT/bench_$name.json') if l.startswith('{')][0])
print('$name driver %.4f ms  headline %.3e' % (d['driver_step']['ms_per_pde_step'], d['value']))"
}
for i in 1 2; do
  run default_$i default
  run nt448_$i nt448
  run g1_$i g1
done
