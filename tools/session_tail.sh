# Tail-split A/B at the bench's 5-step launches: 8 vs 16 half-tile workgroups per XCD band
set -e
mkdir -p gpurun_out
rm -f gpurun_out/tail.jsonl
for i in 1 2 3 4; do
  for t in 8 16; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --tail-split $t | grep '^{' >> gpurun_out/tail.jsonl
  done
done
