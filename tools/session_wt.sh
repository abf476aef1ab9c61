# Write-through packet-state stores (build/wt/libswrt.so, -DSWRT_WT_STORES=1) vs plain: parity subset + bench A/B
set -e
mkdir -p gpurun_out
rm -f gpurun_out/wt.jsonl
SWRT_LIB_PATH=build/wt/libswrt.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "bench_configuration or large_ensemble" > gpurun_out/wt_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 | grep '^{' >> gpurun_out/wt.jsonl
  SWRT_LIB_PATH=build/wt/libswrt.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 | grep '^{' >> gpurun_out/wt.jsonl
done
