cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
SWRT_LIB_PATH=build/variants/pf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "tile or variants or bench or large" > $OUT/pf_parity.log 2>&1; rc=$?; tail -3 $OUT/pf_parity.log; [ $rc -ge 124 ] && exit $rc
bash tools/sweep.sh "" "build/variants/pf.so::" "" "build/variants/pf.so::" "" "build/variants/pf.so::" || exit $?
