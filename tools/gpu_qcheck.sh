#!/bin/bash
# learner / act parity suites + the default bench (no CPU leg)
set -o pipefail
mkdir -p gpurun_out/qcheck
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_qmlp_gpu.py tests/test_learner_golden_gpu.py tests/test_qnet_gpu.py tests/test_draws_gpu.py tests/test_trainer_gpu.py tests/test_qmix_gpu.py tests/test_distributed_gpu.py -m gpu > gpurun_out/qcheck/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/qcheck/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/qcheck/bench.json 2> gpurun_out/qcheck/bench.err
echo "bench rc=$?"; python -c "
import json; d=json.load(open('gpurun_out/qcheck/bench.json')); print(d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms'], d['other_schedule'], d['roofline']['frac'])"
