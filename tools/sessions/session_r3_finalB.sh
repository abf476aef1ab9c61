#!/bin/bash
# Final code, part B: the default bench line, its rocprofv3 kernel trace, QG PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3fb
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
grep '^{' $OUT/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4e ms/step %.4f frac %s driver %.4f' % (d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['driver_step']['ms_per_pde_step']))"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -20 $OUT/bench_prof.err; exit 1; }
bash tools/pmc_qg.sh $OUT/qg || exit $?
