#!/bin/bash
# A/B of a trainer env switch: bash tools/gpu_ab_env.sh VAR  (bench with VAR=0 / 1, twice each)
set -o pipefail
mkdir -p gpurun_out
V=$1
for i in 0 1 2 3; do
  x=$((i % 2))
  env $V=$x timeout -k 10 300 python bench.py --no-cpu --env-steps 0 > gpurun_out/ab_$i.json 2>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/ab_$i.json'))
print('$V=$x', 'value %.3fM' % (d['value'] / 1e6), 'ms %.4f' % d['ms_per_step'], 'env_kernel %.4f' % d['env_step_kernel_ms'], 'learn %.4f' % d['learn_ms'], 'strict %.3fM' % (d['strict_schedule_steps_per_s'] / 1e6))
"
done
