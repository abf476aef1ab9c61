# diagnostic: the host's HIP calls at the end of the drivers' ode23 intervals (tools/o23_end_gap.py)
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r6oe}; mkdir -p $O
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $O/tr -o o -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 16 > $O/bench.log 2>&1 || exit 1
python3 tools/o23_end_gap.py $O/tr --show 4 > $O/end_gap.txt 2>&1; tail -30 $O/end_gap.txt
