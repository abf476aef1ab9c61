#!/bin/bash
# Round 4 final-code measurement: PMC passes of the bench's packet kernel (installed into
# profiles/pmc.json on the box and copied back), the default bench line, and the same command
# under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4m
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_collect.sh $OUT/pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
tail -2 $OUT/pmc.log
python3 tools/pmc_merge.py --install $OUT/pmc/pmc.json && cp profiles/pmc.json $OUT/pmc_installed.json
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/summarize_bench.py $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 > $OUT/bench_under_rocprof.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
python tools/summarize_bench.py $OUT/bench_under_rocprof.json
head -6 $OUT/prof/bench_kernel_stats.csv
