# round 6: the first-step kernel's attached event and the host-observed join at
# the end of split ode23 calls, A/B against SWRT_ODE23_MARKERS=1 (the markers)
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r6om}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ode23.py tests/test_gpu_hazard.py tests/test_dist_gpu.py "tests/test_gpu_qg.py::test_qg2_speculative_steps_bit_identical" -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    SWRT_ODE23_MARKERS=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 32 > $O/ab_${v}_$i.log 2>&1 || exit 1
    python3 -c "
import json,sys
d=json.loads([l for l in open('$O/ab_${v}_$i.log') if l.startswith('{')][-1])['driver_step_ode23']
print('markers=$v run $i', round(d['ms_per_pde_step'],4), d.get('clock_ghz_observed'), d.get('ode23_chained_intervals'), d.get('ode23_per_interval'))
"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o o -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 16 > $O/tr.log 2>&1 || exit 1
f=$(find $O/tr -name "o_kernel_trace.csv")
python3 tools/ode23_timeline.py $f --interval -3 > $O/tl.txt 2>&1
grep -h "interval_us" $O/tl.txt | tail -8
