#!/bin/bash
# Split-tile workgroups at small shard sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3m
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --steps 40"
run() {
  local name=$1; shift
  timeout -k 10 120 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?
  python -c "import json; d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0]); print('$name', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'])"
}
for n in 125000 250000 500000; do
  run u$n --packets $n
  run h$n --packets $n --tail-split 1000 --tail-quarters 0
  run q$n --packets $n --tail-split 0 --tail-quarters 1000
done
run h1000000 --packets 1000000 --tail-split 1000 --tail-quarters 0
run u1000000 --packets 1000000
