cd "${GRAFT_REPO_ROOT}"
bash tools/sweep.sh "--tail-split 0" "--tail-split 128" "--tail-split 64" "--tail-split 16" "--tail-split 0" "--tail-split 128" || exit $?
for ts in 0 128; do
SWRT_LIB_PATH=build/variants/phase.so timeout -k 10 200 python tools/phase_timing.py --samples 8 --tail-split $ts --dump gpurun_out/phase_ts$ts.npz > gpurun_out/phase_ts$ts.log 2>&1 || exit $?
done
