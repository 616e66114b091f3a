#!/bin/bash
# Weight-gradient split-K: ordered partial sums (default) vs f32 atomics (EVX_BWD_ATOMIC=1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qmlp_gpu.py tests/test_qnet_gpu.py tests/test_trainer_gpu.py tests/test_qmix_gpu.py tests/test_prio_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_bwd.log 2>&1 || { tail -40 gpurun_out/t_bwd.log; exit 1; }
tail -3 gpurun_out/t_bwd.log
for i in 0 1 2 3; do
  at=$((i % 2))
  EVX_BWD_ATOMIC=$at timeout -k 10 300 python bench.py --no-cpu --env-steps 0 > gpurun_out/bwd_$i.json 2>gpurun_out/bwd.err || { tail -20 gpurun_out/bwd.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/bwd_$i.json'))
print('atomic=$at', 'value %.3fM' % (d['value'] / 1e6), 'ms %.4f' % d['ms_per_step'], 'env_kernel %.4f' % d['env_step_kernel_ms'], 'learn %.4f' % d['learn_ms'], 'strict %.3fM' % (d['strict_schedule_steps_per_s'] / 1e6))
"
done
