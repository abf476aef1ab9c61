#!/bin/bash
# VALU-issue fraction of the secondary rows' kernels (xka_kernel, spectral
# kernels): one rocprofv3 --pmc pass (SQ_INSTS_VALU, SQ_WAVES, GRBM_GUI_ACTIVE)
# with the kernel trace over tools/bench_rows.py and tools/bench_spectral.py,
# then tools/pmc_kernels.py -> <outdir>/rows_pmc.json.
# usage: tools/pmc_rows.sh <outdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d "$OUT/rows" -o run -- python3 "$ROOT/tools/bench_rows.py" > "$OUT/rows.log" 2>&1 || { tail -5 "$OUT/rows.log"; exit 1; }
timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d "$OUT/spec" -o run -- python3 "$ROOT/tools/bench_spectral.py" --packets 262144 > "$OUT/spec.log" 2>&1 || { tail -5 "$OUT/spec.log"; exit 1; }
python3 tools/pmc_kernels.py "$OUT" > "$OUT/rows_pmc.json"
