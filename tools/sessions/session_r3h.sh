#!/bin/bash
# Driver step vs tile-workgroup size (PDE kernels co-residing with the packet
# launch) and one vs two packet streams; alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r3h
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 40 --ode23-steps 0 --steps 30"
for i in 1 2; do
  for v in base nt384 nt256 ps2; do
    case $v in
      base) env=""; extra="";;
      ps2) env=""; extra="--packet-streams 2";;
      *) env="SWRT_LIB_PATH=$ROOT/build/variants/$v.so"; extra="";;
    esac
    env $env timeout -k 10 200 python bench.py $B $extra > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python -c "import json; d=json.loads([l for l in open('$OUT/bench_${v}_$i.json') if l.startswith('{')][0]); print('$v run $i', '%.4e'%d['value'], 'launch %.4f'%d['roofline']['avg_launch_ms'], 'driver %.4f'%d['driver_step']['ms_per_pde_step'])"
  done
done
