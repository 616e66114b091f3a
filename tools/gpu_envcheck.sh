#!/bin/bash
# env parity tests + stamps (prof build) + env/train bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_dropin_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_env.log 2>&1 || { tail -40 gpurun_out/t_env.log; exit 1; }
tail -1 gpurun_out/t_env.log
EVACX_LIB=libevacx_prof.so timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps_prof.txt 2>&1 || { tail gpurun_out/stamps_prof.txt; exit 1; }
grep -E "groups:|contested|cycles/env-step|launch span|wide  |single-wave  " gpurun_out/stamps_prof.txt
timeout -k 10 300 python bench.py --no-cpu --mode env > gpurun_out/b_env.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --no-cpu --env-steps 0 --strict-steps 0 > gpurun_out/b_tr.json 2>/dev/null || exit 1
python -c "import json;a=json.load(open('gpurun_out/b_env.json'));b=json.load(open('gpurun_out/b_tr.json'));print('env-mode kernel %.4f value %.3fM | train value %.3fM ms %.4f kernel %.4f' % (a['env_step_kernel_ms'], a['value']/1e6, b['value']/1e6, b['ms_per_step'], b['env_step_kernel_ms']))"
