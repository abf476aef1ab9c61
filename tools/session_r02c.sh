cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_qg.py -x -v --timeout 300 --timeout-method thread -k "512" > $OUT/qg512.log 2>&1; rc=$?; tail -5 $OUT/qg512.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python tools/fp32_study.py > $OUT/fp32_study.json 2> $OUT/fp32_study.err; rc=$?; echo "fp32 rc=$rc"; tail -c 3000 $OUT/fp32_study.json; [ $rc -ne 0 ] && { tail $OUT/fp32_study.err; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1500 $OUT/bench.log
