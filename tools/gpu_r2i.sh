#!/bin/bash
# lib A/B (global-scratch bitmaps on every grid) + per-config bench lines (cfg2, cfg4 conv, cfg5 prio) + cfg4 kernel trace
set -o pipefail
O=gpurun_out/r2i; mkdir -p $O
bash tools/gpu_libab.sh dqn-marl_amd/evacx/libevacx_bigg.so || exit $?
timeout -k 10 300 python bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 > $O/b_cfg2.json 2>$O/b_cfg2.err || { tail -5 $O/b_cfg2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 > $O/b_cfg5.json 2>$O/b_cfg5.err || { tail -5 $O/b_cfg5.err; exit 1; }
timeout -k 10 500 python bench.py --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 20 --other-steps 0 --start-steps 0 --batch 1024 > $O/b_cfg4.json 2>$O/b_cfg4.err || { tail -5 $O/b_cfg4.err; exit 1; }
for c in cfg2 cfg5 cfg4; do python -c "import json;d=json.load(open('$O/b_$c.json'));print('$c value %.3fM env-steps/s, ms %.3f, env kernel %.3f ms, frac %.3f, env-only %s' % (d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['roofline']['frac'], d.get('env_only_steps_per_s')))"; done
bash tools/gpu_cfg4prof.sh
