#!/bin/bash
# Round 4 start: smoke, GPU suite, default bench line on the unchanged round-3 tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
grep '^{' $OUT/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4e ms/step %.4f frac %s driver %.4f' % (d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['driver_step']['ms_per_pde_step'])); print(json.dumps(d.get('strong_scaling_forecast')))"
