#!/bin/bash
# GPU-box A/B session:
#   tools/gpu_ab.sh <outdir> <name>=<lib|default>[@<extra bench args, commas for spaces>] ... -- <bench.py args>
# runs bench.py once per variant (library via SWRT_LIB_PATH, plus its extra
# arguments), alternating the variants twice, each run under its own time
# limit; a crash or timeout ends the session.  Lines go to <outdir>/<name>_<i>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
names=(); libs=(); extras=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  spec=$1; names+=("${spec%%=*}"); rest=${spec#*=}
  libs+=("${rest%%@*}")
  if [[ $rest == *@* ]]; then extras+=("${rest#*@}"); else extras+=(""); fi
  shift
done
shift
for rep in 1 2; do
  for i in "${!names[@]}"; do
    lib=${libs[$i]}; [ "$lib" = default ] && lib=""
    extra=${extras[$i]//,/ }
    echo "== ${names[$i]} rep $rep: $* $extra"
    SWRT_LIB_PATH=$lib timeout -k 10 300 python bench.py "$@" $extra > "$OUT/${names[$i]}_$rep.json" \
      2> >(tee "$OUT/${names[$i]}_$rep.err" >&2)
    rc=$?
    echo "rc=$rc"; tail -c 300 "$OUT/${names[$i]}_$rep.json"; echo
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${names[$i]}_$rep.err"; exit $rc; fi
  done
done
