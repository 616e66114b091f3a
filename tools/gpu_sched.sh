#!/bin/bash
# Scheduling check: env/trainer/prio/drop-in GPU tests, gap probe, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_trainer_gpu.py tests/test_prio_gpu.py tests/test_dropin_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sched.log 2>&1 || { tail -40 gpurun_out/t_sched.log; exit 1; }
tail -2 gpurun_out/t_sched.log
bash tools/gpu_gap.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b_train.json 2>gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/b_train.json"))
print("value %.3fM" % (d["value"] / 1e6), "ms %.4f" % d["ms_per_step"], "env_kernel %.4f" % d["env_step_kernel_ms"],
      "learn", d.get("learn_ms"), "strict", d.get("strict_schedule_steps_per_s"), "env_only", d.get("env_only_steps_per_s"), "loss", d.get("last_loss"))
PY
