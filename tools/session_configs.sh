# The other BASELINE configs (parity cases, not bench lines): configs[1] 256^2 1e4 steady, configs[2] 512^2 1e5 blend
set -e
mkdir -p gpurun_out
rm -f gpurun_out/configs.jsonl
timeout -k 10 120 python bench.py --no-cpu-baseline --nx 256 --packets 10000 --mode steady --steps 100 | grep '^{' >> gpurun_out/configs.jsonl
timeout -k 10 120 python bench.py --no-cpu-baseline --nx 256 --packets 10000 --mode steady --steps 20 --substeps 64 --rebin-every 64 | grep '^{' >> gpurun_out/configs.jsonl
timeout -k 10 120 python bench.py --no-cpu-baseline --nx 512 --packets 100000 --steps 100 | grep '^{' >> gpurun_out/configs.jsonl
timeout -k 10 120 python bench.py --no-cpu-baseline --nx 512 --packets 100000 --steps 25 --intervals 4 | grep '^{' >> gpurun_out/configs.jsonl
