#!/bin/bash
# Round 4: column pass fused with the Jacobian (2-layer QG); full GPU suite, bench x2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 400 python bench.py --no-cpu-baseline --no-fma --forecast-intervals 1 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -20 $OUT/bench_$i.err; exit 1; }
python tools/summarize_bench.py $OUT/bench_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 5 --driver-steps 40 > $OUT/drv.json 2> $OUT/drv.err || { tail -5 $OUT/drv.err; exit 1; }
python tools/driver_trace_summary.py $OUT/prof/run_kernel_trace.csv --steps 40 > $OUT/drv_summary.txt
cat $OUT/drv_summary.txt
