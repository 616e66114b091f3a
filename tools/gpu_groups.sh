#!/bin/bash
# Grouped-trainer check: split/group GPU tests, then the bench at 1, 2 and 4 env groups.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_trainer_gpu.py -x -q --timeout 200 --timeout-method thread -k "split or groups or schedules or order_ahead or runs_and_learns" > gpurun_out/t_groups.log 2>&1 || { tail -40 gpurun_out/t_groups.log; exit 1; }
tail -2 gpurun_out/t_groups.log
for g in 1 2 4; do
  timeout -k 10 300 python bench.py --no-cpu --groups $g --env-steps 0 > gpurun_out/b_g$g.json 2>gpurun_out/b_g$g.err || { tail -20 gpurun_out/b_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_g$g.json'));print('groups $g value %.3fM ms %.4f env_kernel %.4f learn %.4f strict %.3fM' % (d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms'], d['strict_schedule_steps_per_s']/1e6))"
done
