#!/bin/bash
# envs per workgroup at the 32768-env workload: 4 (heavy workgroups + light waves) vs 1 / 2 (no heavy path)
set -o pipefail
mkdir -p gpurun_out/nwb
for N in 4 1 2; do
  EVX_STEP_NWB=$N timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --other-steps 0 --start-steps 10 \
      > gpurun_out/nwb/n$N.json 2> gpurun_out/nwb/n$N.err || exit $?
  python - "$N" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/nwb/n{sys.argv[1]}.json"))
print(sys.argv[1], round(d["value"] / 1e6, 3), "env_ms", round(d["env_step_kernel_ms"], 3),
      "envonly", round(d["env_only_steps_per_s"] / 1e6, 2), "start", round(d["start_phase"]["steps_per_s"] / 1e6, 3),
      "start_env_ms", round(d["start_phase"]["env_step_kernel_ms"], 3), flush=True)
PY
done
