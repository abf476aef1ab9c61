cd "${GRAFT_REPO_ROOT}"
for P in 500000 1000000; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 30 --warmup 3 --packets $P --no-cpu-baseline > gpurun_out/b2_$P.log 2>&1 || exit $?
grep '^{' gpurun_out/b2_$P.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("2 ranks", d["config"]["packets_per_gpu"], "%.4g"%d["value"], "launch %.1f"%(d["roofline"]["avg_launch_ms"]*1e3))'
done
timeout -k 10 300 python bench.py --no-cpu-baseline --packets 2000000 > gpurun_out/b1_2M.log 2>&1 || exit $?
grep '^{' gpurun_out/b1_2M.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("1 rank", d["config"]["packets_per_gpu"], "%.4g"%d["value"], "launch %.1f"%(d["roofline"]["avg_launch_ms"]*1e3))'
