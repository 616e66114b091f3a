#!/bin/bash
# round 5: backward GEMM LDS-fragment prefetch A/B (libevacx_qzq.so): x3 learn parity, then per-kernel times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5tn; mkdir -p $OUT
cd $R
EVX_LIB=$R/dqn-marl_amd/evacx/libevacx_qzq.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_bench_scale_gpu.py -k "x3_learn" tests/test_learner_golden_gpu.py tests/test_qmlp_x3_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/tests.log | head -30; exit $rc; }
TAGS="default qzq default qzq" bash tools/gpu_r5_tn.sh
