#!/bin/bash
# HBM traffic of the hot kernel from PMC counters: separate rocprofv3 passes for
# FETCH_SIZE and WRITE_SIZE (they do not fit one TCC pass on gfx950), kernel
# trace only (no sys/runtime trace beside --pmc).  Then tools/pmc_parse.py
# writes per-launch bytes into profiles/traffic.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run -- python3 "$ROOT/bench.py" $BENCH_ARGS > "$OUT/$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$C.log"; exit $rc; fi
done
python3 tools/pmc_parse.py "$OUT" $BENCH_ARGS
