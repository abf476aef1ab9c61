#!/bin/bash
# spectral kernel A/B: tools/pmc_rows.sh once per build (SWRT_LIB_PATH)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in "$@"; do
  n=$(basename $lib .so)
  SWRT_LIB_PATH=$lib bash tools/pmc_rows.sh gpurun_out/spec_$n || exit $?
done
