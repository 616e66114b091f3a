set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_prio_gpu.py tests/test_env_gpu.py -x -v --timeout 200 --timeout-method thread -k "prio or cfg4 or cfg5" > gpurun_out/t_prio.log 2>&1 || { tail -40 gpurun_out/t_prio.log; exit 1; }
tail -8 gpurun_out/t_prio.log
timeout -k 10 300 python bench.py --no-cpu --replay prioritized > gpurun_out/b_prio.json 2> gpurun_out/b_prio.err || { tail -20 gpurun_out/b_prio.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 --env-steps 0 > gpurun_out/b_cfg5.json 2> gpurun_out/b_cfg5.err || { tail -20 gpurun_out/b_cfg5.err; exit 1; }
python - <<'PY'
import json
for f in ["gpurun_out/b_prio.json", "gpurun_out/b_cfg5.json"]:
    d = json.load(open(f))
    print(f, "value %.3fM" % (d["value"] / 1e6), "ms %.4f" % d["ms_per_step"], "env_kernel %.4f" % d["env_step_kernel_ms"],
          "learn", d.get("learn_ms"), "strict", d.get("strict_schedule_steps_per_s"), "env_only", d.get("env_only_steps_per_s"), "loss", d.get("last_loss"))
PY
