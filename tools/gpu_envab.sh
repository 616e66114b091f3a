#!/bin/bash
# env parity suites + the default bench (no CPU leg) for an env_step_kernel change
set -o pipefail
mkdir -p gpurun_out/envab
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_env_gpu.py tests/test_layoutset_gpu.py tests/test_trainer_gpu.py -m gpu > gpurun_out/envab/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/envab/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/envab/bench.json 2> gpurun_out/envab/bench.err
echo "bench rc=$?"; cat gpurun_out/envab/bench.json
