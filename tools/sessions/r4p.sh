#!/bin/bash
# Round 4: re-binning every 5 / 10 / 20 steps at the shard sizes and 1e6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4p
mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --steps 100"
for n in 125000 250000 1000000; do
for r in 20 10 5 20 10; do
timeout -k 10 120 python bench.py --packets $n --rebin-every $r $Q > $OUT/n${n}_r$r.json 2>> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$OUT/n${n}_r$r.json') if l.startswith('{')][-1]); print('$n rebin $r %.4e' % d['value'])"
done
done
