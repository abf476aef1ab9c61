# Upper bound of a multi-interval launch: 10 (and 20) steps per launch vs the bench's 5
set -e
mkdir -p gpurun_out
rm -f gpurun_out/ls.jsonl
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 | grep '^{' >> gpurun_out/ls.jsonl
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --substeps 10 | grep '^{' >> gpurun_out/ls.jsonl
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --substeps 20 | grep '^{' >> gpurun_out/ls.jsonl
done
