#!/bin/bash
# backward GEMM change: learn parity tests, then the learn-chain profile (tools/gpu_learnprof.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/learn2; mkdir -p $OUT
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_qmlp_gpu.py \
   tests/test_bench_scale_gpu.py -k "learn or backward or grad or x3" > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
bash tools/gpu_learnprof.sh ${1:-b}
