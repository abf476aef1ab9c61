#!/bin/bash
# A/B session: GPU parity, bench sweep of variants, rocprofv3 kernel stats of the product build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ode23.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep.sh "$@" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o ab --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_ab.log 2>&1
echo "prof rc=$?"
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_ab/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:70]:70s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:8.2f} pct {float(r['Percentage']):6.2f}")
PY
