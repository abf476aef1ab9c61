# QG stream priority A/B: high (default) vs normal priority vs one stream, alternating
set -e
mkdir -p gpurun_out
rm -f gpurun_out/pipe_ab.jsonl
for i in 1 2; do
  timeout -k 10 120 python tools/bench_pipeline.py >> gpurun_out/pipe_ab.jsonl
  SWRT_QG_PRIO=0 timeout -k 10 120 python tools/bench_pipeline.py >> gpurun_out/pipe_ab.jsonl
  timeout -k 10 120 python tools/bench_pipeline.py --one-stream >> gpurun_out/pipe_ab.jsonl
done
