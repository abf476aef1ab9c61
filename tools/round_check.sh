#!/bin/bash
# Full check: smoke + GPU tests + default bench + rocprof stats + 2-rank bench (gloo, shared GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_run.sh all || exit $?
OUT=gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 3 --gather > $OUT/bench_2rank.log 2>&1
rc=$?; echo "2-rank bench rc=$rc"; grep '^{' $OUT/bench_2rank.log | cut -c1-400
exit 0
