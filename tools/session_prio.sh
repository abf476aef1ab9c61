cd "${GRAFT_REPO_ROOT}"
bash tools/sweep.sh "" "build/variants/prio.so::" "" "build/variants/prio.so::" "" "build/variants/prio.so::" "build/variants/prio.so::--tail-split 0" "--tail-split 0" || exit $?
SWRT_LIB_PATH=build/variants/phaseprio.so timeout -k 10 200 python tools/phase_timing.py --samples 8 --dump gpurun_out/phase_prio.npz > gpurun_out/phase_prio.log 2>&1 || exit $?
SWRT_LIB_PATH=build/variants/phaseprio.so timeout -k 10 200 python tools/phase_timing.py --samples 8 --tail-split 0 --dump gpurun_out/phase_prio0.npz > gpurun_out/phase_prio0.log 2>&1 || exit $?
