#!/bin/bash
# Packet streams 1 vs 2 across ensemble sizes (512^2 blend; 256^2 steady at 1e4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3af
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --driver-steps 0"
run() {
  local name=$1; shift
  timeout -k 10 200 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0])
print('$name %.4e  ms/step %.4f' % (d['value'], d['ms_per_step']))"
}
for n in 30000 62500 125000 250000 500000; do
  for s in 1 2; do
    run n${n}_s$s --packets $n --packet-streams $s --steps 100
  done
done
