# QG post-step kernels fused (one spectra launch, Jacobian + CFL max): GPU tests + pipeline timing
set -e
mkdir -p gpurun_out
rm -f gpurun_out/pipe_ab.jsonl
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_qg.py tests/test_gpu_parity.py > gpurun_out/qg_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python tools/bench_pipeline.py >> gpurun_out/pipe_ab.jsonl
done
