#!/bin/bash
# Round 4: kernel trace of the metric phase at 1.25e5 packets (re-binning cost per cycle).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t125k -o run -- python3 bench.py --packets 125000 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --steps 40 --warmup 4 > $OUT/t125k.json 2> $OUT/t125k.err || { tail -5 $OUT/t125k.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t125k1 -o run -- python3 bench.py --packets 125000 --packet-streams 1 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --steps 40 --warmup 4 > $OUT/t125k1.json 2> $OUT/t125k1.err || { tail -5 $OUT/t125k1.err; exit 1; }
echo done
