#!/bin/bash
# Full GPU check of the in-tree build: all GPU tests, the bench line, the
# driver pipeline with ode23, a kernel trace of the bench.  Stops at the first
# crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || exit $?
grep '^{' $OUT/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench %.4g  launch %.1f us  driver %.3f ms" % (d["value"], d["roofline"]["avg_launch_ms"]*1e3, d["driver_step"]["ms_per_pde_step"]))'
timeout -k 10 300 python tools/bench_pipeline.py --ode23 > $OUT/pipeline.json 2>&1 || exit $?
tail -1 $OUT/pipeline.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --driver-steps 0 > $OUT/prof.log 2>&1 || exit $?
head -3 $OUT/prof/bench_kernel_stats.csv
