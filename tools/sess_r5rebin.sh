#!/bin/bash
# Round-5: the ode23 re-binning period with the stage-1 chain (every 1 / 2 / 3
# calls: build/var/rb1.so, the default library, build/var/rb3.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--steps 1 --warmup 0 --no-cpu-baseline --no-forecast --no-fma --driver-steps 0 --ode23-steps 13"
timeout -k 10 900 bash tools/gpu_ab.sh r5rebin rb2=default rb1=build/var/rb1.so rb3=build/var/rb3.so -- $A \
  > gpurun_out/r5rebin.log 2>&1 || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5rebin/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    o = d["driver_step_ode23"]
    print(f, round(o["ms_per_pde_step"], 4), o.get("ode23_chained_intervals"), round(o.get("clock_ghz_observed") or 0, 3))
PY
