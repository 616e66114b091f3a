#!/bin/bash
# env.step occupancy experiment: default build vs builds with __launch_bounds__ min waves per EU 3 / 4.
set -o pipefail
mkdir -p gpurun_out
for v in "" w3 w4 "" w3 w4; do
  lib=""
  [ -n "$v" ] && lib="$PWD/dqn-marl_amd/evacx/libevacx_$v.so"
  EVX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --strict-steps 0 > gpurun_out/occ.json 2>gpurun_out/occ.err || { tail -20 gpurun_out/occ.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/occ.json'))
print('${v:-w2}', 'value %.3fM' % (d['value'] / 1e6), 'ms %.4f' % d['ms_per_step'], 'env_kernel %.4f' % d['env_step_kernel_ms'], 'env_only %.3fM' % (d['env_only_steps_per_s'] / 1e6))
"
done
