#!/bin/bash
# GPU check used during development: env parity tests, then env-mode and train benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_env_gpu.py tests/test_dropin_gpu.py tests/test_trainer_gpu.py -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 300 python bench.py --no-cpu --mode env > gpurun_out/b_env.json 2>gpurun_out/b.err || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b_train.json 2>>gpurun_out/b.err || exit 1
python - <<'PY'
import json
for f in ["gpurun_out/b_env.json", "gpurun_out/b_train.json"]:
    d = json.load(open(f))
    print(f, "value %.3fM" % (d["value"] / 1e6), "ms %.4f" % d["ms_per_step"], "env_kernel %.4f" % d["env_step_kernel_ms"],
          "learn", d.get("learn_ms"), "strict", d.get("strict_schedule_steps_per_s"), "env_only", d.get("env_only_steps_per_s"))
PY
