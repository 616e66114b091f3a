#!/bin/bash
# env parity suites + bench + stamp probe at 32768 envs
set -o pipefail
mkdir -p gpurun_out/envq
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py tests/test_layoutset_gpu.py tests/test_dropin_gpu.py -m gpu > gpurun_out/envq/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/envq/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 > gpurun_out/envq/bench.json 2> gpurun_out/envq/bench.err || exit $?
python -c "
import json; d=json.load(open('gpurun_out/envq/bench.json')); print(d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms'], d['env_only_steps_per_s']/1e6, d['start_phase']['env_step_kernel_ms'], d['roofline']['frac'])"
timeout -k 10 300 python tools/stamp_probe.py --envs 32768 > gpurun_out/envq/stamps.txt 2>&1
echo "stamps rc=$?"; grep -v Warn gpurun_out/envq/stamps.txt | tail -14
