#!/bin/bash
# A/B of the act fast path (static pre-activation table) on one box: bench with it off / on / off / on.
set -o pipefail
mkdir -p gpurun_out
for i in 0 1 2 3; do
  s=$((i % 2))
  EVX_ACT_STATIC=$s timeout -k 10 300 python bench.py --no-cpu --env-steps 0 --strict-steps 0 > gpurun_out/ab_$i.json 2>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/ab_$i.json'))
print('static=$s', 'value %.3fM' % (d['value'] / 1e6), 'ms %.4f' % d['ms_per_step'], 'env_kernel %.4f' % d['env_step_kernel_ms'], 'act', d.get('act_kernel_ms'), 'learn', d.get('learn_ms'))
"
done
