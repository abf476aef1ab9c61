#!/bin/bash
# Kernel traces of the driver step: HEAD's QG FFT kernels vs the new ones.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3r
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 10 --driver-steps 40"
for v in head new; do
  if [ $v = head ]; then export SWRT_LIB_PATH=$PWD/build_ab/libswrt_head.so; else unset SWRT_LIB_PATH; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o run -- python3 bench.py $B > $OUT/$v.json 2> $OUT/$v.err || exit $?
  python tools/timeline.py $OUT/$v/run_kernel_trace.csv --launches 80 > $OUT/$v.timeline.txt || exit $?
  tail -25 $OUT/$v.timeline.txt
done
