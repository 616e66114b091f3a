#!/bin/bash
# The other BASELINE configs as bench lines (1 GPU, per-GPU shares): cfg2, cfg4 (conv Q-net), cfg5
set -o pipefail
mkdir -p gpurun_out
#timeout -k 10 300 python bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 --env-steps 0 > gpurun_out/b_cfg2.json 2>gpurun_out/b_cfg2.err || { tail -5 gpurun_out/b_cfg2.err; exit 1; }
#timeout -k 10 300 python bench.py --no-cpu --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 --env-steps 0 > gpurun_out/b_cfg5.json 2>gpurun_out/b_cfg5.err || { tail -5 gpurun_out/b_cfg5.err; exit 1; }
timeout -k 10 500 python bench.py --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 20 --other-steps 0 --start-steps 0 --batch 1024 > gpurun_out/b_cfg4.json 2>gpurun_out/b_cfg4.err || { tail -5 gpurun_out/b_cfg4.err; exit 1; }
for c in cfg4; do python -c "import json;d=json.load(open('gpurun_out/b_$c.json'));print('$c value %.3fM env-steps/s, %.1fM agent-transitions/s, ms %.3f, env kernel %.3f ms, env-only %s' % (d['value']/1e6, d['agent_transitions_per_s']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d.get('env_only_steps_per_s')))"; done
