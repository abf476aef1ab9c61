#!/bin/bash
# Four packet streams: stream tests, then bench A/B (1 / 2 / 4 streams), one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3aa
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_qg.py -x -q --timeout 200 --timeout-method thread -k "packet_streams" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --driver-steps 40"
for i in 1 2 3; do
  for s in 2 4 1; do
    timeout -k 10 200 python bench.py $B --packet-streams $s > $OUT/bench_s${s}_$i.json 2> $OUT/bench_s${s}_$i.err || { tail -5 $OUT/bench_s${s}_$i.err; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('$OUT/bench_s${s}_$i.json') if l.startswith('{')][0])
print('streams $s run $i: %.4e  ms/step %.4f driver %.4f' % (d['value'], d['ms_per_step'], d['driver_step']['ms_per_pde_step']))"
  done
done
