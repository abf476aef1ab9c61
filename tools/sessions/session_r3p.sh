#!/bin/bash
# A/B on one box: HEAD's QG FFT kernels (build_ab/libswrt_head.so) vs the
# grouped FFT kernels (in-tree build): QG-only step and the driver step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 10 --driver-steps 40"
for i in 1 2; do
  for v in head new; do
    if [ $v = head ]; then export SWRT_LIB_PATH=$PWD/build_ab/libswrt_head.so; else unset SWRT_LIB_PATH; fi
    timeout -k 10 60 python tools/bench_qg.py > $OUT/qg_${v}_$i.json 2>/dev/null || exit $?
    timeout -k 10 200 python bench.py $B > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python -c "
import json
q=json.loads([l for l in open('$OUT/qg_${v}_$i.json') if l.startswith('{')][0])
d=json.loads([l for l in open('$OUT/bench_${v}_$i.json') if l.startswith('{')][0])
print('$v $i qg %.4f ms  driver %.4f ms  headline %.3e' % (q['ms_per_step'], d['driver_step']['ms_per_pde_step'], d['value']))"
  done
done
unset SWRT_LIB_PATH
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qgtrace -o run -- python3 tools/bench_qg.py > $OUT/qgtrace.log 2>&1 || exit $?
