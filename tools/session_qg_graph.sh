# A/B of hipGraph replay of the QG step (tools/bench_pipeline.py), alternating
set -e
mkdir -p gpurun_out
rm -f gpurun_out/pipe_ab.jsonl
for i in 1 2; do
  timeout -k 10 120 python tools/bench_pipeline.py --qg-graphs >> gpurun_out/pipe_ab.jsonl
  timeout -k 10 120 python tools/bench_pipeline.py >> gpurun_out/pipe_ab.jsonl
done
