cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_mex_gateway.py tests/test_gpu_spectral.py tests/test_gpu_qg.py -x -v --timeout 300 --timeout-method thread -k "mex or gateway or ode23_packets_gpu or config5 or integrator_substitution or two_schemes or spectral_and_qg or ode_symplectic_gpu" > $OUT/new_tests.log 2>&1; rc=$?; tail -15 $OUT/new_tests.log; exit $rc
