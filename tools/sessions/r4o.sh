#!/bin/bash
# Round 4: small-shard launch-parameter sweep at 1.25e5 / 2.5e5 packets (re-binning cadence, tail split, streams).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4o
mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --steps 100"
for n in 125000 250000; do
for opt in "--rebin-every 20" "--rebin-every 40" "--rebin-every 60" "--tail-split 8" "--tail-split 32" "--packet-streams 1" "--packet-streams 4" "--rebin-every 20"; do
tag=$(echo "$n $opt" | tr ' -' '__')
timeout -k 10 120 python bench.py --packets $n $opt $Q > $OUT/$tag.json 2>> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$OUT/$tag.json') if l.startswith('{')][-1]); print('$n $opt %.4e' % d['value'])"
done
done
