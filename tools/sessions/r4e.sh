#!/bin/bash
# Round 4: ode23 attempt kernel without scratch spills (bits, interval time, PMC); driver-step kernel trace at a 1.25e5 shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ode23.py tests/test_mex_gateway.py tests/test_gpu_qg.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_ode23.log 2>&1 || { tail -30 $OUT/pytest_ode23.log; exit 1; }
tail -1 $OUT/pytest_ode23.log
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 6 > $OUT/ode23_$i.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$OUT/ode23_$i.json') if l.startswith('{')][-1]); print('ode23 interval %.4f ms' % d['driver_step_ode23']['ms_per_pde_step'])"
done
bash tools/pmc_ode23.sh $OUT/ode23_pmc > $OUT/ode23_pmc.log 2>&1 || { tail -20 $OUT/ode23_pmc.log; exit 1; }
tail -1 $OUT/ode23_pmc.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof125k -o run -- python3 bench.py --packets 125000 --no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --steps 5 --driver-steps 40 > $OUT/drv125k.json 2> $OUT/drv125k.err || { tail -5 $OUT/drv125k.err; exit 1; }
python tools/driver_trace_summary.py $OUT/prof125k/run_kernel_trace.csv --steps 40 --timeline 2 > $OUT/drv125k_summary.txt
head -60 $OUT/drv125k_summary.txt
