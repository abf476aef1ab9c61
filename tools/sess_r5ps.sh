#!/bin/bash
# Round-5: the leapfrog driver step with the packet launch split over 2
# streams (default) or 1 (--packet-streams 1), at 1e6 and at the 8-GPU shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--steps 10 --warmup 2 --no-cpu-baseline --no-forecast --no-fma --ode23-steps 0 --driver-steps 100"
timeout -k 10 600 bash tools/gpu_ab.sh r5ps/1m ps2=default ps1=default@--packet-streams,1 -- $A > gpurun_out/r5ps_1m.log 2>&1 &&
timeout -k 10 600 bash tools/gpu_ab.sh r5ps/125k ps2=default ps1=default@--packet-streams,1 -- $A --packets 125000 \
  > gpurun_out/r5ps_125k.log 2>&1 || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5ps/*/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, "value", round(d["value"] / 1e10, 4), "drv", round(d["driver_step"]["ms_per_pde_step"], 4))
PY
