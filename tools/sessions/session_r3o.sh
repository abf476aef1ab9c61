#!/bin/bash
# QG FFT kernels with every global load issued up front: GPU tests, QG-only
# timing and kernel trace, driver step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 60 python tools/bench_qg.py > $OUT/qg_time.json 2>&1 || exit $?
cat $OUT/qg_time.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qgtrace -o run -- python3 tools/bench_qg.py > $OUT/qgtrace.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][0]); print('value %.3e'%d['value'], {k: d[k] for k in d if 'driver' in k})"
