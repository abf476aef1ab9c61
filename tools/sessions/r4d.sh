#!/bin/bash
# Round 4: sparse-tile launch A/B at strong-scaling shard sizes, then smoke, GPU suite, default bench, ode23 PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4d
mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0"
for n in 125000 250000 500000; do
  for sp in 1 2 1 2; do
    timeout -k 10 120 python bench.py --packets $n --sparse-tiles $sp $Q > $OUT/ab_${n}_sp${sp}.json 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_${n}_sp${sp}.json') if l.startswith('{')][-1]); print('$n sp$sp %.4e %.4f ms' % (d['value'], d['roofline']['launch_span_ms']))"
  done
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/summarize_bench.py $OUT/bench.json
bash tools/pmc_ode23.sh $OUT/ode23_pmc > $OUT/ode23_pmc.log 2>&1 || { tail -20 $OUT/ode23_pmc.log; exit 1; }
tail -3 $OUT/ode23_pmc.log
