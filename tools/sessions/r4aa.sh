#!/bin/bash
# Round 4 final tree: kernel traces of the end-to-end driver step at 1e6
# packets and at the 8-GPU shard (1.25e5), per-kernel summaries and timelines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4aa
mkdir -p $OUT
export TMPDIR=/tmp
for N in 1000000 125000; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/d$N -o run -- python3 bench.py --packets $N --no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 5 --driver-steps 40 > $OUT/d$N.json 2> $OUT/d$N.err || { tail -5 $OUT/d$N.err; exit 1; }
python tools/driver_trace_summary.py $OUT/d$N/run_kernel_trace.csv --steps 40 > $OUT/d${N}_summary.txt
python tools/driver_trace_summary.py $OUT/d$N/run_kernel_trace.csv --steps 40 --timeline 3 > $OUT/d${N}_timeline.txt
head -12 $OUT/d${N}_summary.txt
done
