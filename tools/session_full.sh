#!/bin/bash
# Round evidence: smoke, GPU tests, default bench, rocprofv3 kernel stats,
# 2-rank bench, C-ABI CLI, PMC traffic + SQ counters of the default config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/round_check.sh || exit $?
OUT=gpurun_out
timeout -k 10 200 ./build/bin/swrt_cli > $OUT/cli.log 2>&1; echo "cli rc=$?"; cat $OUT/cli.log | tail -2
bash tools/pmc_traffic.sh > $OUT/pmc_traffic.log 2>&1; echo "pmc traffic rc=$?"; tail -2 $OUT/pmc_traffic.log
bash tools/pmc_counters.sh "--steps 10 --warmup 2 --no-cpu-baseline" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES" "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" > $OUT/pmc_sq.log 2>&1; echo "pmc sq rc=$?"; tail -9 $OUT/pmc_sq.log
exit 0
