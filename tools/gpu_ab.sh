#!/bin/bash
# GPU-box A/B session: `tools/gpu_ab.sh <outdir> <name>=<lib or "default"> ... -- <bench.py args>`
# runs bench.py once per variant library (SWRT_LIB_PATH), alternating the
# variants twice, each run under its own time limit; a crash or timeout ends
# the session.  Lines go to <outdir>/<name>_<i>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
names=(); libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("${1%%=*}"); libs+=("${1#*=}"); shift; done
shift
for rep in 1 2; do
  for i in "${!names[@]}"; do
    lib=${libs[$i]}; [ "$lib" = default ] && lib=""
    echo "== ${names[$i]} rep $rep: $*"
    SWRT_LIB_PATH=$lib timeout -k 10 300 python bench.py "$@" > "$OUT/${names[$i]}_$rep.json" 2> >(tee "$OUT/${names[$i]}_$rep.err" >&2)
    rc=$?
    echo "rc=$rc"; tail -c 600 "$OUT/${names[$i]}_$rep.json"; echo
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${names[$i]}_$rep.err"; exit $rc; fi
  done
done
