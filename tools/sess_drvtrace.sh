# round 6: kernel + HIP API trace of the leapfrog driver step (TwoLayerLoop, 1e6 packets)
export TMPDIR=/tmp
O=gpurun_out/r6drv; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/tr -o d -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fma --no-forecast --driver-steps 60 --ode23-steps 0 > $O/b.log 2>&1; echo rc=$?
