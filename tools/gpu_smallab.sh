#!/bin/bash
# learner-kernel parity suites, then cfg2 / cfg5 training-step A/B over libevacx_<tag>.so builds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_qmlp_gpu.py tests/test_qmlp_x3_gpu.py tests/test_qnet_gpu.py tests/test_target_table_gpu.py tests/test_trainer_gpu.py \
    tests/test_learner_golden_gpu.py tests/test_draws_gpu.py > gpurun_out/smallcheck.log 2>&1
rc=$?; tail -2 gpurun_out/smallcheck.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/smallcheck.log | head -30; exit $rc; }
bash tools/gpu_cfgab.sh "$1"
