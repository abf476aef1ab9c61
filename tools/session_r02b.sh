cd "${GRAFT_REPO_ROOT}"
bash tools/pmc_collect.sh gpurun_out/pmc "--steps 12 --warmup 2 --no-cpu-baseline" || exit $?
python3 tools/pmc_merge.py --install gpurun_out/pmc/pmc.json || exit $?
bash tools/sweep.sh "" "--tail-split 0" "" "--tail-split 0" "--tail-split 8" "" "--tail-split 0" || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
