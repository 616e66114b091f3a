#!/bin/bash
# MLP fast-path check: numerics tests, trainer tests, microbenchmark, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qmlp_gpu.py tests/test_qnet_gpu.py tests/test_trainer_gpu.py tests/test_prio_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_qmlp.log 2>&1 || { tail -40 gpurun_out/t_qmlp.log; exit 1; }
tail -3 gpurun_out/t_qmlp.log
timeout -k 10 200 python tools/qmlp_bench.py > gpurun_out/qmlp_bench.log 2>&1 || { tail -20 gpurun_out/qmlp_bench.log; exit 1; }
cat gpurun_out/qmlp_bench.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b_train.json 2>gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/b_train.json"))
print("value %.3fM" % (d["value"] / 1e6), "ms %.4f" % d["ms_per_step"], "env_kernel %.4f" % d["env_step_kernel_ms"],
      "learn", d.get("learn_ms"), "strict", d.get("strict_schedule_steps_per_s"), "env_only", d.get("env_only_steps_per_s"), "loss", d.get("last_loss"))
PY
