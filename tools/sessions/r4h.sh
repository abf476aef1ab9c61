#!/bin/bash
# Round 4: speculative PDE steps in TwoLayerLoop (bits + driver step at 1e6 and the shard sizes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_qg.log 2>&1 || { tail -30 $OUT/pytest_qg.log; exit 1; }
tail -1 $OUT/pytest_qg.log
for i in 1 2; do
timeout -k 10 400 python bench.py --no-cpu-baseline --no-fma --ode23-steps 0 --forecast-intervals 1 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -20 $OUT/bench_$i.err; exit 1; }
python tools/summarize_bench.py $OUT/bench_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/h125000 -o run -- python3 bench.py --packets 125000 --no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 5 --driver-steps 40 > $OUT/h125000.json 2> $OUT/h125000.err || { tail -5 $OUT/h125000.err; exit 1; }
python tools/driver_host_timeline.py $OUT/h125000 --steps 3 > $OUT/h125000_timeline.txt
python tools/driver_trace_summary.py $OUT/h125000/run_kernel_trace.csv --steps 40 > $OUT/h125000_summary.txt
head -3 $OUT/h125000_summary.txt
