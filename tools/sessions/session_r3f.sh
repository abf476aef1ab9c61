#!/bin/bash
# GPU tests, then one vs two packet streams (bench line), the two-rank upper
# bound, and the driver pipeline with its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/r3f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B="--no-cpu-baseline --no-forecast --no-fma --driver-steps 20 --ode23-steps 0"
for ps in 1 2 1 2; do
  timeout -k 10 200 python bench.py --packet-streams $ps $B > $OUT/bench_ps$ps.json 2> $OUT/bench_ps$ps.err || exit $?
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_ps$ps.json') if l.startswith('{')][0]); print('ps=$ps', '%.4e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'driver %.4f'%d['driver_step']['ms_per_pde_step'])"
done
timeout -k 10 200 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 > $OUT/bench_2rank.json 2> $OUT/bench_2rank.err || exit $?
python -c "import json; d=json.loads([l for l in open('$OUT/bench_2rank.json') if l.startswith('{')][0]); print('2rank', '%.4e'%d['value'], d['n_gpus'], d['config']['packets_per_gpu'])"
timeout -k 10 120 python tools/bench_pipeline.py > $OUT/pipeline.json 2> $OUT/pipeline.err || exit $?
cat $OUT/pipeline.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pipe_prof -o pipe \
  -- python3 $ROOT/tools/bench_pipeline.py > $OUT/pipe_prof.log 2>&1 || exit $?
echo done
