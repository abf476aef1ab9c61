# Kernel trace of the driver pipeline (two streams) for the overlap analysis
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptrace -o pipe -- python3 tools/bench_pipeline.py --steps 20 > gpurun_out/ptrace.log 2>&1
