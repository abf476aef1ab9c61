# Driver pipeline: GPU tests (QG, intervals) + A/B of grouped packet intervals (4 vs 1 per call)
set -e
mkdir -p gpurun_out
rm -f gpurun_out/pipe_ab.jsonl
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_qg.py tests/test_gpu_intervals.py > gpurun_out/qg_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python tools/bench_pipeline.py >> gpurun_out/pipe_ab.jsonl
  timeout -k 10 120 python tools/bench_pipeline.py --intervals 1 >> gpurun_out/pipe_ab.jsonl
done
