#!/bin/bash
# The other BASELINE configs on the final code (parity cases, not bench lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3ad
mkdir -p $OUT
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --driver-steps 0 --steps 100"
run() {
  local name=$1; shift
  timeout -k 10 200 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0])
print('$name %.4e  ms/step %.4f' % (d['value'], d['ms_per_step']))"
}
run cfg1_steady_256_1e4 --nx 256 --packets 10000 --mode steady
run cfg1_steady_256_1e4_64steps --nx 256 --packets 10000 --mode steady --substeps 64
run cfg2_blend_512_1e5 --packets 100000
run cfg2_blend_512_1e5_iv4 --packets 100000 --intervals 4
run cfg3_blend_512_1e6_iv4 --intervals 4
