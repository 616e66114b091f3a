#!/bin/bash
# A/B of act builds: libevacx.so vs libevacx_b.so (EVX_LIB), the act microbench at 524288 rows
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=$R/dqn-marl_amd/evacx
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_qmlp_x3_gpu.py::test_x3_persistent_act_matches_64_row_kernel" 2>&1 | tail -2 || exit 1
for i in 1 2; do
  for lib in libevacx.so libevacx_b.so; do
    echo -n "$lib: "; EVX_LIB=$L/$lib timeout -k 10 120 python tools/act3_bench.py --table-frac 1.0 2>&1 | tail -1 || exit 1
  done
done
