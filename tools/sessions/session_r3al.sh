#!/bin/bash
# Packet streams on a CU mask leaving k CUs to the QG stream (diagnostic build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3al
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 20 --driver-steps 40"
run() {
  local name=$1 lib=$2 res=$3
  if [ $lib = default ]; then unset SWRT_LIB_PATH; else export SWRT_LIB_PATH=$PWD/build_ab/libswrt_cumask.so; fi
  export SWRT_DIAG_RESERVE=$res
  timeout -k 10 200 python bench.py $B > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0])
print('$name driver %.4f ms  headline %.3e' % (d['driver_step']['ms_per_pde_step'], d['value']))"
}
for i in 1 2; do
  run def_$i default none
  run low8_$i cumask low:8
  run str8_$i cumask stride:8
  run str16_$i cumask stride:16
  run low32_$i cumask low:32
done
