#!/bin/bash
# Round 4: uneven shares of the two packet streams (SWRT_DEBUG_STREAM_SPLIT)
# — bits (calls queued back to back), then an in-box A/B at 1e6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4ad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -k "stream_split or packet_streams" -m gpu -x -v --timeout 100 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
for sk in 0 5 6 3; do
timeout -k 10 200 python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 0 --stream-split $sk > $OUT/sk${sk}_$i.json 2> $OUT/sk${sk}_$i.err || { tail -20 $OUT/sk${sk}_$i.err; exit 1; }
echo "stream_split=$sk run $i $(python tools/summarize_bench.py $OUT/sk${sk}_$i.json | head -1)"
done
done
