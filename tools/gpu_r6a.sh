#!/bin/bash
# round 6, first box: the tests the ADVICE fixes touch, cfg3's counter record, the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_trainer_gpu.py \
  tests/test_order_gpu.py tests/test_env_gpu.py::test_order_ahead_and_obs_double_buffer_do_not_change_results \
  tests/test_layoutset_gpu.py > gpurun_out/r6a_tests.log 2>&1 || { tail -30 gpurun_out/r6a_tests.log; exit 1; }
tail -3 gpurun_out/r6a_tests.log
bash tools/gpu_r6_counters.sh cfg3 > gpurun_out/r6a_cnt.log 2>&1 || { tail -20 gpurun_out/r6a_cnt.log; exit 1; }
cp gpurun_out/r6cnt/env_counters_stationary_cfg3.json profiles/r6/
cd $R && timeout -k 10 500 python bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || { tail gpurun_out/r6a_bench.err; exit 1; }
cat gpurun_out/r6a_bench.json
