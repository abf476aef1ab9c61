#!/bin/bash
# Re-binning cadence with two packet streams (20 default vs 40 / 30).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3ah
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --driver-steps 0 --steps 80"
for i in 1 2 3; do
  for r in 20 40 30; do
    timeout -k 10 200 python bench.py $B --rebin-every $r > $OUT/r${r}_$i.json 2> $OUT/r${r}_$i.err || { tail -5 $OUT/r${r}_$i.err; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('$OUT/r${r}_$i.json') if l.startswith('{')][0])
print('rebin $r run $i: %.4e  ms/step %.4f' % (d['value'], d['ms_per_step']))"
  done
done
