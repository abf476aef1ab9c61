# Multi-interval launches: parity tests, then bench A/B (1, 2, 4 PDE intervals per call)
set -e
mkdir -p gpurun_out
rm -f gpurun_out/iv.jsonl
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_intervals.py tests/test_gpu_parity.py > gpurun_out/iv_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 | grep '^{' >> gpurun_out/iv.jsonl
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --intervals 2 | grep '^{' >> gpurun_out/iv.jsonl
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --intervals 4 | grep '^{' >> gpurun_out/iv.jsonl
done
