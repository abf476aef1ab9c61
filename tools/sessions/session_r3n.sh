#!/bin/bash
# Per-packet kernel and 8x8 tiles at small shard sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3n
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --steps 40"
run() {
  local name=$1; shift
  timeout -k 10 120 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?
  python -c "import json; d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0]); print('$name', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'])"
}
for n in 125000 250000; do
  run k1_$n --packets $n --kernel 1
  run t8_$n --packets $n --tile 8
done
