#!/bin/bash
# Spatial-shard diagnostic, y-bands (tiles spread over every XCD band).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3l
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --packets 125000 --steps 40"
run() {
  local name=$1; shift
  timeout -k 10 120 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?
  python -c "import json; d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0]); print('$name', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'])"
}
run uniform
run yband --positions yband
run yband_q --positions yband --tail-split 0 --tail-quarters 1000
run yband_h --positions yband --tail-split 1000 --tail-quarters 0
run yband4 --positions yband --band-parts 4 --packets 250000
run yband4_h --positions yband --band-parts 4 --packets 250000 --tail-split 1000 --tail-quarters 0
run yband2 --positions yband --band-parts 2 --packets 500000
