# Multi-interval bench (4 PDE intervals per call): bench line + rocprofv3 kernel stats
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python bench.py --intervals 4 --steps 12 --warmup 2 --cpu-seconds 5 | grep '^{' > gpurun_out/iv4_bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iv4prof -o iv4 -- python3 bench.py --intervals 4 --steps 12 --warmup 2 --no-cpu-baseline > gpurun_out/iv4_prof.log 2>&1
