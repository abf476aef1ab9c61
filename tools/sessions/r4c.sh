#!/bin/bash
# Round 4: smoke, GPU suite, bench with the new forecasts (intervals, driver step at shard sizes), ode23 PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/summarize_bench.py $OUT/bench.json
bash tools/pmc_ode23.sh $OUT/ode23_pmc > $OUT/ode23_pmc.log 2>&1 || { tail -20 $OUT/ode23_pmc.log; exit 1; }
tail -3 $OUT/ode23_pmc.log
