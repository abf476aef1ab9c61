# round 6: device-scope release on the ordering events (A/B against SWRT_EVENT_SYSTEM=1), suite first
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r6ev}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  for v in 0 1; do
    SWRT_EVENT_SYSTEM=$v timeout -k 10 400 python bench.py --no-cpu-baseline --no-fma --no-forecast > $O/ab_${v}_$i.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$O/ab_${v}_$i.log') if l.startswith('{')][-1])
print('system=$v run $i value %.4g clk %.3f driver %.4f ode23 %.4f' % (d['value'], d['roofline']['clock_ghz_observed'] or 0, d['driver_step']['ms_per_pde_step'], d['driver_step_ode23']['ms_per_pde_step']))
"
  done
done
