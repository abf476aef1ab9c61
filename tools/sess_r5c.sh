# driver step: the PDE on its own stream beside the packets vs serialised on
# the packet stream (packet-free kernel shapes), at the shard sizes of 8/4/2 GPUs
export SESSION=r5c
for n in 125000 250000 500000; do
  timeout -k 10 900 bash tools/gpu_ab.sh r5c/n$n sep=default@--qg-stream,1 ser=default@--qg-stream,0 -- \
    --packets $n --steps 20 --no-forecast --no-cpu-baseline --no-fma --driver-steps 100 --ode23-steps 0 || exit $?
done
