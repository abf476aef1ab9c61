#!/bin/bash
# A/B on one box: HEAD vs grouped FFT kernels with global / LDS twiddles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3s
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 10 --driver-steps 40"
run() {
  local name=$1 lib=$2 grp=$3 split=$4 twg=$5
  if [ $lib = head ]; then export SWRT_LIB_PATH=$PWD/build_ab/libswrt_head.so; else unset SWRT_LIB_PATH; fi
  export SWRT_FFT_GROUP=$grp SWRT_POST_SPLIT=$split SWRT_TW_GLOBAL=$twg
  timeout -k 10 60 python tools/bench_qg.py > $OUT/qg_$name.json 2>/dev/null || exit $?
  timeout -k 10 200 python bench.py $B > $OUT/bench_$name.json 2> $OUT/bench_$name.err || exit $?
  python -c "
import json
q=json.loads([l for l in open('$OUT/qg_$name.json') if l.startswith('{')][0])
d=json.loads([l for l in open('$OUT/bench_$name.json') if l.startswith('{')][0])
print('$name qg %.4f ms  driver %.4f ms  headline %.3e' % (q['ms_per_step'], d['driver_step']['ms_per_pde_step'], d['value']))"
}
run head_a head 4 1 0
run g1s0_glob new 1 0 1
run g1s0_lds new 1 0 0
run g4s1_glob new 4 1 1
run g4s1_lds new 4 1 0
run g4s0_glob new 4 0 1
run head_b head 4 1 0
run g1s0_glob_b new 1 0 1
