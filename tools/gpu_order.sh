#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_trainer_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_order.log 2>&1 || { tail -30 gpurun_out/t_order.log; exit 1; }
tail -2 gpurun_out/t_order.log
for i in 0 1; do
  timeout -k 10 300 python bench.py --no-cpu --env-steps 0 > gpurun_out/bo_$i.json 2>gpurun_out/bo.err || { tail -20 gpurun_out/bo.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/bo_$i.json'))
print('value %.3fM' % (d['value'] / 1e6), 'ms %.4f' % d['ms_per_step'], 'env_kernel %.4f' % d['env_step_kernel_ms'], 'strict %.3fM' % (d['strict_schedule_steps_per_s'] / 1e6))
"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_order" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --no-cpu --env-steps 0 --strict-steps 0 > "$R/gpurun_out/prof_order.log" 2>&1 || exit 1
f=$(find "$R/gpurun_out/prof_order" -name "*kernel_stats.csv" | head -1)
grep -E "env_order|qact|env_step_kernel" "$f" | cut -c1-200
