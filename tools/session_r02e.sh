cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -6 $OUT/pytest_gpu.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 3 --gather --driver-steps 10 > $OUT/bench_2rank.log 2>&1; rc=$?; echo "2rank rc=$rc"; grep '^{' $OUT/bench_2rank.log | cut -c1-300
exit 0
