#!/bin/bash
# Spatial-shard diagnostic: 1.25e5 packets confined to 1/8 of the domain (the
# density a y-band shard of 8 GPUs would hold), whole tiles vs quarter-tile
# workgroups, vs the index shard (uniform positions).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3j
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --packets 125000 --steps 40"
run() {
  local name=$1; shift
  timeout -k 10 120 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?
  python -c "import json; d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0]); print('$name', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'])"
}
run uniform
run band --positions band
run band_q --positions band --tail-split 0 --tail-quarters 1000
run band_h --positions band --tail-split 1000 --tail-quarters 0
run band_1s --positions band --packet-streams 1
run band_q1s --positions band --tail-split 0 --tail-quarters 1000 --packet-streams 1
run uniform_1e6 --packets 1000000
