# Driver pipeline with a fixed dt (the 1-layer driver's loop): grouped packet intervals 4 vs 1
set -e
mkdir -p gpurun_out
rm -f gpurun_out/pipe_ab.jsonl
for i in 1 2; do
  timeout -k 10 120 python tools/bench_pipeline.py --fixed-dt --intervals 4 --steps 40 >> gpurun_out/pipe_ab.jsonl
  timeout -k 10 120 python tools/bench_pipeline.py --fixed-dt --intervals 1 --steps 40 >> gpurun_out/pipe_ab.jsonl
done
