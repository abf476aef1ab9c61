#!/bin/bash
# Final code (FFT grouping by co-run), part A again: smoke, GPU suite, tile PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3fc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/pmc_collect.sh $OUT/pmc > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
bash tools/pmc_collect.sh $OUT/pmc_fma "--steps 12 --warmup 2 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --packet-streams 1 --gather-mode 1" > $OUT/pmc_fma.log 2>&1 || { tail $OUT/pmc_fma.log; exit 1; }
python tools/pmc_merge.py --install $OUT/pmc/pmc.json && python tools/pmc_merge.py --install $OUT/pmc_fma/pmc.json && cp profiles/pmc.json $OUT/pmc_installed.json || exit 1
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
grep '^{' $OUT/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4e ms/step %.4f frac %s driver %.4f' % (d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['driver_step']['ms_per_pde_step']))"
