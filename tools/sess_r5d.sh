# spatial vs index partition: bit-exactness of the 8x8-tile shards, then the
# strong-scaling and driver forecasts of both
export SESSION=r5d
OUT=gpurun_out/r5d; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "spatial_shard or small_shard" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/gpu_ab.sh r5d/ab spatial=default@--partition,spatial index=default@--partition,index -- \
  --no-cpu-baseline --no-fma --forecast-intervals 1 --driver-steps 50 --forecast-driver-steps 60 --ode23-steps 0
