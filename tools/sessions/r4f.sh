#!/bin/bash
# Round 4: host/device timeline of the driver step (kernel + HIP API trace) at 1.25e5 and 1e6 packets.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4f
mkdir -p $OUT
export TMPDIR=/tmp
for n in 125000 1000000; do
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/h$n -o run -- python3 bench.py --packets $n --no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 5 --driver-steps 40 > $OUT/h$n.json 2> $OUT/h$n.err || { tail -5 $OUT/h$n.err; exit 1; }
python tools/driver_host_timeline.py $OUT/h$n --steps 3 > $OUT/h${n}_timeline.txt
tail -45 $OUT/h${n}_timeline.txt
done
