#!/bin/bash
# Round-5 session q: step_packet_xka without scratch (row weights shifted
# through registers).  xka tests, then tools/bench_rows.py alternating the
# previous and the new library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rsw.py tests/test_gpu_parity.py -k "xka" -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in new head; do
    lib=""; [ $v = head ] && lib=build/var/head.so
    SWRT_LIB_PATH=$lib timeout -k 10 200 python tools/bench_rows.py > $O/rows_${v}_$rep.json 2> $O/rows_${v}_$rep.err || exit $?
    python -c "import json; j=json.loads(open('$O/rows_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', j['xka'])"
  done
done
