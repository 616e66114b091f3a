#!/bin/bash
# env_step iteration: env parity suites, then per-phase stamps and a short bench line (cfg3)
set -o pipefail
mkdir -p gpurun_out/envit
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_env_gpu.py tests/test_bench_scale_gpu.py tests/test_dropin_gpu.py tests/test_layoutset_gpu.py \
    tests/test_order_gpu.py tests/test_trainer_gpu.py > gpurun_out/envit/tests.log 2>&1
rc=$?; tail -3 gpurun_out/envit/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/envit/tests.log | head -20; exit $rc; }
timeout -k 10 300 python tools/stamp_probe.py --envs 32768 > gpurun_out/envit/stamps.txt 2>&1 || exit 1
grep -v Warning gpurun_out/envit/stamps.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --start-steps 0 > gpurun_out/envit/bench.json 2> gpurun_out/envit/bench.err || { tail gpurun_out/envit/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/envit/bench.json')); print('value', d['value']/1e6, 'ms', d['ms_per_step'], 'env', d['env_step_kernel_ms'], 'learn', d['learn_ms'], 'env_only', d['env_only_steps_per_s']/1e6)"
