#!/bin/bash
# One stream below 65,536 packets: GPU suite, small configs, default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3ag
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="--no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --driver-steps 0"
run() {
  local name=$1; shift
  timeout -k 10 200 python bench.py $B "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][0])
print('$name %.4e  ms/step %.4f' % (d['value'], d['ms_per_step']))"
}
run cfg1_sub5 --nx 256 --packets 10000 --mode steady --steps 200
run cfg1_sub64 --nx 256 --packets 10000 --mode steady --substeps 64 --steps 50
run n30000 --packets 30000 --steps 100
run cfg2 --packets 100000 --steps 100
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
grep '^{' $OUT/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default value %.4e ms/step %.4f frac %s driver %.4f' % (d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['driver_step']['ms_per_pde_step']))"
