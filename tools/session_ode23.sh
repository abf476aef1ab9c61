# ode23 fused attempt: GPU ode23 tests + the pipeline's ode23 interval timing
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ode23.py > gpurun_out/ode23_tests.log 2>&1
timeout -k 10 200 python tools/bench_pipeline.py --ode23 > gpurun_out/pipe_ode23.json
