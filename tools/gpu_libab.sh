#!/bin/bash
# A/B of experiment library builds (EVX_LIB) on the default bench: usage tools/gpu_libab.sh lib1.so lib2.so ...
# (the in-tree libevacx.so first, as the control)
set -o pipefail
mkdir -p gpurun_out/libab
for L in dqn-marl_amd/evacx/libevacx.so "$@" dqn-marl_amd/evacx/libevacx.so; do
  T=$(basename $L .so)
  EVX_LIB=$(pwd)/$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --other-steps 0 --start-steps 10 \
      > gpurun_out/libab/$T.json 2> gpurun_out/libab/$T.err || exit $?
  python - "gpurun_out/libab/$T.json" "$T" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sp = d.get("start_phase") or {}
print(sys.argv[2], round(d["value"] / 1e6, 3), "env_ms", round(d["env_step_kernel_ms"], 3),
      "envonly", round((d.get("env_only_steps_per_s") or 0) / 1e6, 2), "start", round((sp.get("steps_per_s") or 0) / 1e6, 3),
      "start_env_ms", round(sp.get("env_step_kernel_ms") or 0, 3), flush=True)
PY
done
