#!/bin/bash
# x3 conv GEMM: learner numerics (f32 and x3 conv vs torch, golden learner) then the cfg4 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_qnet_gpu.py tests/test_learner_golden_gpu.py > gpurun_out/x3conv_tests.log 2>&1 || { tail -30 gpurun_out/x3conv_tests.log; exit 1; }
tail -3 gpurun_out/x3conv_tests.log
bash tools/gpu_configs.sh
