# diagnostic: the ode23 driver step's HIP API calls beside its kernels (host timeline between intervals)
export TMPDIR=/tmp
O=gpurun_out/r6o23api; mkdir -p $O
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $O/tr -o o -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 16 > $O/bench.log 2>&1; echo "rc=$?"
ls -R $O/tr | head
python3 tools/o23_api_gap.py $O/tr > $O/gap.txt 2>&1; tail -5 $O/gap.txt
