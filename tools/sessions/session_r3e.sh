#!/bin/bash
# (1) two concurrent half-ensembles on one GPU (2 ranks, gloo): the upper bound
#     of splitting the packet launch over two streams; (2) the driver pipeline
#     and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r3e
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0"
timeout -k 10 200 python bench.py --gpus 2 --dist-backend gloo $B > $OUT/bench_2rank.json 2> $OUT/bench_2rank.err || exit $?
echo "2rank: $(cat $OUT/bench_2rank.json | cut -c1-120)"
timeout -k 10 120 python bench.py $B > $OUT/bench_1rank.json 2> $OUT/bench_1rank.err || exit $?
echo "1rank: $(cat $OUT/bench_1rank.json | cut -c1-120)"
timeout -k 10 120 python tools/bench_pipeline.py > $OUT/pipeline.json 2> $OUT/pipeline.err || exit $?
cat $OUT/pipeline.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pipe_prof -o pipe \
  -- python3 $ROOT/tools/bench_pipeline.py > $OUT/pipe_prof.log 2>&1 || exit $?
echo done
