#!/bin/bash
# rocprofv3 kernel stats of the end-to-end driver step (PDE + snapshots + packets)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe -o pipe --output-format csv -- python3 tools/bench_pipeline.py --steps 20 $PIPE_ARGS > gpurun_out/prof_pipe.log 2>&1
echo "prof rc=$?"
grep '^{' gpurun_out/prof_pipe.log | cut -c1-400
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_pipe/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:80]:80s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:8.2f} tot_ms {float(r['TotalDurationNs'])/1e6:8.3f}")
PY
