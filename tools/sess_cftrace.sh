# round 6: kernel traces of the ode23 driver step with and without the chained first attempt
export TMPDIR=/tmp
O=gpurun_out/r6cft; mkdir -p $O
for v in 1 0; do
  SWRT_ODE23_CHAIN_FIRST=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$v -o o -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 16 > $O/b$v.log 2>&1 || exit 1
  f=$(find $O/tr$v -name "o_kernel_trace.csv")
  python3 tools/ode23_timeline.py $f --interval -3 --json $O/tl$v.json > $O/tl$v.txt 2>&1
  python3 tools/ode23_timeline.py $f --interval -2 >> $O/tl$v.txt 2>&1
  echo "== chain_first=$v"; grep -h "interval_us" $O/tl$v.txt | tail -12
done
