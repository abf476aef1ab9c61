#!/bin/bash
# Round 4 final tree: smoke, the full GPU suite, PMC of the bench's packet
# kernel (installed on the box, copied back) and of the 1.25e5 shard in both
# launch shapes, the default bench line, and the bench under
# rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/pmc_collect.sh $OUT/pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
tail -2 $OUT/pmc.log
python3 tools/pmc_merge.py --install $OUT/pmc/pmc.json && cp profiles/pmc.json $OUT/pmc_installed.json
for sp in 1 2; do
bash tools/pmc_collect.sh $OUT/pmc125k_sp$sp "--packets 125000 --steps 40 --warmup 4 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --packet-streams 1 --sparse-tiles $sp" > $OUT/pmc125k_sp$sp.log 2>&1 || { tail -20 $OUT/pmc125k_sp$sp.log; exit 1; }
tail -1 $OUT/pmc125k_sp$sp.log
done
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/summarize_bench.py $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 > $OUT/bench_under_rocprof.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
python tools/summarize_bench.py $OUT/bench_under_rocprof.json
head -6 $OUT/prof/bench_kernel_stats.csv
