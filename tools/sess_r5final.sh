#!/bin/bash
# Round-5 evidence session: smoke, the default bench line (what the driver
# runs), the same command's metric phase under rocprofv3 --kernel-trace
# --stats.  usage: tools/sess_r5final.sh <outdir under gpurun_out>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r5final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- \
  python3 bench.py --no-cpu-baseline --driver-steps 0 --ode23-steps 0 --no-fma --no-forecast \
  > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || { tail -5 $O/bench_under_rocprof.err; exit 1; }
echo prof done
