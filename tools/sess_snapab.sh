export TMPDIR=/tmp
O=gpurun_out/r6snap2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_qg.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_qg.log 2>&1; echo "pytest rc=$?"; tail -2 $O/pytest_qg.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o rx -- python3 tools/owner_legs.py --receiver 142857 --owner --steps 100 > $O/legs_tr.log 2>&1 && python3 tools/timeline.py $(find $O/tr -name "rx_kernel_trace.csv") --match tile_leapfrog --launches 60 > $O/timeline.txt 2>&1; echo "trace rc=$?"; cat $O/timeline.txt | head -30
timeout -k 10 300 python3 tools/owner_legs.py --receiver 142857 333333 --owner 0 --steps 200 > $O/legs.log 2>&1; echo "legs rc=$?"; grep -v "^{" $O/legs.log | tail -4
