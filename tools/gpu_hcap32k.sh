#!/bin/bash
# heavy-envs cap sweep at the 32768-env workload: stationary (headline) and start phase
set -o pipefail
mkdir -p gpurun_out/hcap
for C in 176 512 1024 2048 4096; do
  EVX_HEAVY_CAP=$C timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --other-steps 0 --start-steps 10 \
      > gpurun_out/hcap/c$C.json 2> gpurun_out/hcap/c$C.err || exit $?
  python - "$C" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/hcap/c{sys.argv[1]}.json"))
print(sys.argv[1], round(d["value"] / 1e6, 3), "env_ms", round(d["env_step_kernel_ms"], 3),
      "envonly", round(d["env_only_steps_per_s"] / 1e6, 2), "start", round(d["start_phase"]["steps_per_s"] / 1e6, 3),
      "start_env_ms", round(d["start_phase"]["env_step_kernel_ms"], 3), flush=True)
PY
done
