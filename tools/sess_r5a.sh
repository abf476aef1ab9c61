export SESSION=r5a
export PHASE_LIBS="phase phase128"
export AB_VARIANTS="def=default sp128=build/var/sp128.so"
export AB_ARGS="--packets 125000 --steps 40 --no-forecast --no-cpu-baseline --no-fma --driver-steps 100 --ode23-steps 0"
bash tools/gpu_run.sh test bench prof phase ab
