# round 6: the ode23 chain with the first step and first attempt queued too
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r6cf}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ode23.py tests/test_gpu_hazard.py "tests/test_gpu_qg.py::test_qg2_speculative_steps_bit_identical" -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  for v in 1 0; do
    SWRT_ODE23_CHAIN_FIRST=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fma --no-forecast --driver-steps 0 --ode23-steps 16 > $O/ab_${v}_$i.log 2>&1 || exit 1
    python3 -c "
import json,sys
d=json.loads([l for l in open('$O/ab_${v}_$i.log') if l.startswith('{')][-1])['driver_step_ode23']
print('chain_first=$v run $i', round(d['ms_per_pde_step'],4), d.get('clock_ghz_observed'), d.get('ode23_chained_intervals'), d.get('ode23_per_interval'))
"
  done
done
