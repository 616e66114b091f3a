#!/bin/bash
# envs per workgroup (EVX_STEP_NWB 4 vs 1) across env counts and configs: where the heavy-env
# workgroups stop paying (latency-bound small launches vs throughput-bound large ones)
set -o pipefail
mkdir -p gpurun_out/nwb2
run() {  # tag nwb args...
  local T=$1 N=$2; shift 2
  EVX_STEP_NWB=$N timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --other-steps 0 "$@" \
      > gpurun_out/nwb2/$T.n$N.json 2> gpurun_out/nwb2/$T.n$N.err || exit $?
  python - "gpurun_out/nwb2/$T.n$N.json" "$T nwb=$N" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sp = d.get("start_phase") or {}
print(sys.argv[2], round(d["value"] / 1e6, 3), "env_ms", round(d["env_step_kernel_ms"], 3),
      "envonly", round((d.get("env_only_steps_per_s") or 0) / 1e6, 2), "start", round((sp.get("steps_per_s") or 0) / 1e6, 3),
      "start_env_ms", round(sp.get("env_step_kernel_ms") or 0, 3), flush=True)
PY
}
for E in 4096 8192 16384; do
  for N in 4 1; do run cfg3e$E $N --envs $E --start-steps 10; done
done
for N in 4 1; do run cfg2 $N --grid 64 --people 569 --robots 8 --envs 4096 --start-steps 10; done
for N in 4 1; do run cfg5 $N --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 --start-steps 0; done
