#!/bin/bash
# Round-5 session e: 384-thread sparse shape (3 waves/SIMD, VGPRs left for the
# PDE's waves) forced at 1e6 and 1.25e5, driver step beside the PDE; then a
# kernel trace of the drivers' ode23 intervals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-cpu-baseline --no-fma --no-forecast --ode23-steps 0 --steps 40"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5e/ode23 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e/ode23 -o ode23 --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 6 --steps 5 \
  > gpurun_out/r5e/ode23/bench.json 2> gpurun_out/r5e/ode23/bench.err &&
timeout -k 10 560 bash tools/gpu_ab.sh r5e/1m def=default sp1=build/var/sp384p1.so@--sparse-tiles,2 \
  sp2=build/var/sp384p2.so@--sparse-tiles,2 -- $A --packets 1000000 &&
timeout -k 10 560 bash tools/gpu_ab.sh r5e/125k def=default sp1=build/var/sp384p1.so@--sparse-tiles,2 \
  sp2=build/var/sp384p2.so@--sparse-tiles,2 -- $A --packets 125000
