#!/bin/bash
# round 6: the persistent x3 act -- bit identity against the 64-row kernel, then the microbench (both kernels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_qmlp_x3_gpu.py::test_x3_persistent_act_matches_64_row_kernel" > gpurun_out/r6b_tests.log 2>&1 || { tail -40 gpurun_out/r6b_tests.log; exit 1; }
tail -5 gpurun_out/r6b_tests.log
for k in "" "--kernel64" ""; do
  timeout -k 10 120 python tools/act3_bench.py --table-frac 1.0 $k 2>&1 | tail -1 || exit 1
done
timeout -k 10 120 python tools/act3_bench.py --table-frac 1.0 --drop-p 0 2>&1 | tail -1 || exit 1
timeout -k 10 200 python tools/act3p_stamps.py
