#!/bin/bash
# F3 suites + the per-robot-nets bench variant (cfg3 workload, strict)
set -o pipefail
mkdir -p gpurun_out/f3
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_qgroup_gpu.py tests/test_draws_gpu.py -m gpu > gpurun_out/f3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/f3/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --start-steps 0 --env-steps 0 --nets per_robot > gpurun_out/f3/bench_per_robot.json 2> gpurun_out/f3/bench_per_robot.err
echo "bench rc=$?"; python -c "
import json; d=json.load(open('gpurun_out/f3/bench_per_robot.json')); print(d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms'], d['last_loss'])"
