# round 6: split leapfrog launches fork only after other packet-stream work (A/B against SWRT_FORK_ALWAYS=1), suite first
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r6fork}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
for i in 1 2 3; do
  for v in 0 1; do
    SWRT_FORK_ALWAYS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-fma --driver-steps 0 --ode23-steps 0 > $O/ab_${v}_$i.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$O/ab_${v}_$i.log') if l.startswith('{')][-1])
ss=d.get('strong_scaling_forecast',{})
print('fork_always=$v run $i value %.4g clk %.3f per-GHz %.4g  G8 %.4g (%.3f)' % (d['value'], d['roofline']['clock_ghz_observed'], d['value']/d['roofline']['clock_ghz_observed'], ss.get('8',{}).get('value_1gpu',0), ss.get('8',{}).get('clock_ghz_observed') or 0))
"
  done
done
