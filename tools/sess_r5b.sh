export SESSION=r5b
bash tools/gpu_run.sh test bench
