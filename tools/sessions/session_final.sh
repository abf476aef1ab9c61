#!/bin/bash
# Round evidence on the in-tree build: smoke, all GPU tests, the default bench
# line, its rocprofv3 kernel trace (metric phase), the PMC passes of the tile
# kernel, the rows (xka, spectral) PMC and the driver pipeline with ode23.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/session_full.sh || exit $?
bash tools/pmc_collect.sh $OUT/pmc "--steps 12 --warmup 2 --no-cpu-baseline --driver-steps 0" || exit $?
bash tools/pmc_rows.sh $OUT/pmcrows || exit $?
# two ranks sharing the GPU (gloo): the multi-process bench path, the device
# gather of the trajectories and the driver phase
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 3 --gather --driver-steps 10 \
  > $OUT/bench_2rank.log 2>&1 || { tail -5 $OUT/bench_2rank.log; exit 1; }
grep '^{' $OUT/bench_2rank.log | cut -c1-200
