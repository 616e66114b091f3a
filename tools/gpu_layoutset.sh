#!/bin/bash
# Per-env layouts (LayoutSet): new parity tests, env/MLP regressions, bench (single-layout path unchanged).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_layoutset_gpu.py tests/test_env_gpu.py tests/test_qmlp_gpu.py tests/test_dropin_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_ls.log 2>&1 || { tail -40 gpurun_out/t_ls.log; exit 1; }
tail -3 gpurun_out/t_ls.log
timeout -k 10 300 python bench.py --no-cpu --strict-steps 0 > gpurun_out/b_ls.json 2>gpurun_out/b_ls.err || { tail -20 gpurun_out/b_ls.err; exit 1; }
python -c "
import json; d = json.load(open('gpurun_out/b_ls.json'))
print('value %.3fM' % (d['value'] / 1e6), 'ms %.4f' % d['ms_per_step'], 'env_kernel %.4f' % d['env_step_kernel_ms'], 'env_only %.3fM' % (d['env_only_steps_per_s'] / 1e6))
"
