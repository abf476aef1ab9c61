#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/gap; mkdir -p $OUT
export TMPDIR=/tmp
for v in "" "--one-stream" "--timing-every 5" "--one-stream --timing-every 5"; do
  timeout -k 10 120 python tools/gap_probe.py $v || exit $?
done
i=0
for v in "" "--one-stream"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$i -o run -- python3 tools/gap_probe.py $v > $OUT/t$i.log 2>&1 || exit $?
done
