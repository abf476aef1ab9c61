#!/bin/bash
# configs[1] (256^2, 1e4 packets, steady): packet streams 1 vs 2, 5 and 64 steps per call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3ae
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --driver-steps 0 --steps 200 --nx 256 --packets 10000 --mode steady"
run() {
  local name=$1; shift
  timeout -k 10 200 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0])
print('$name %.4e  ms/step %.4f' % (d['value'], d['ms_per_step']))"
}
for i in 1 2; do
run s2_sub5_$i --packet-streams 2
run s1_sub5_$i --packet-streams 1
run s2_sub64_$i --packet-streams 2 --substeps 64
run s1_sub64_$i --packet-streams 1 --substeps 64
done
