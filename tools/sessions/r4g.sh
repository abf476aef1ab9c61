#!/bin/bash
# Round 4: re-binning before the snapshot wait, two-plane post-rows beside packets, ode23 packets sorted in place;
# ode23 + QG + parity subset tests, bench, driver traces at 1.25e5 / 1e6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/summarize_bench.py $OUT/bench.json
for n in 125000 1000000; do
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/h$n -o run -- python3 bench.py --packets $n --no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 5 --driver-steps 40 > $OUT/h$n.json 2> $OUT/h$n.err || { tail -5 $OUT/h$n.err; exit 1; }
python tools/driver_host_timeline.py $OUT/h$n --steps 3 > $OUT/h${n}_timeline.txt
python tools/driver_trace_summary.py $OUT/h$n/run_kernel_trace.csv --steps 40 > $OUT/h${n}_summary.txt
head -12 $OUT/h${n}_summary.txt
done
