cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep.sh "" "" "" || exit $?
bash tools/pmc_collect.sh gpurun_out/pmc "--steps 12 --warmup 2 --no-cpu-baseline --driver-steps 0" || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --steps 50 --driver-steps 0 > $OUT/prof.log 2>&1; echo "prof rc=$?"
