cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_ode23.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_13.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_13.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_pipeline.py --ode23 --steps 5 > gpurun_out/pipe_new_$i.log 2>&1 || exit $?
  SWRT_LIB_PATH=build/variants/old.so timeout -k 10 200 python tools/bench_pipeline.py --ode23 --steps 5 > gpurun_out/pipe_old_$i.log 2>&1 || exit $?
done
for f in gpurun_out/pipe_*_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["step_ms"],4), {k: round(v,4) for k,v in d["ode23"].items()})')"; done
