cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/pmc_traffic.sh || exit $?
bash tools/pmc_counters.sh "--steps 10 --warmup 2 --no-cpu-baseline" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES" "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" || exit $?
SWRT_LIB_PATH=build/variants/phase.so timeout -k 10 200 python tools/phase_timing.py --samples 8 > gpurun_out/phase.log 2>&1; echo phase rc=$?
