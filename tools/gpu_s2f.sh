#!/bin/bash
# round 6 (session 2): qbwd3 dZ2 staged in LDS (16-B stores): learn parity, cfg2 / cfg5 / cfg3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2f; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_scale_gpu.py \
  tests/test_qmlp_x3_gpu.py tests/test_qmlp_gpu.py tests/test_trainer_gpu.py tests/test_learner_golden_gpu.py \
  tests/test_qgroup_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- --grid 64 --people 569 --robots 8 --envs 4096 2>&1 | tee $O/ab_cfg2.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- --robots 32 --envs 8192 --replay prioritized --replay-capacity 4194304 2>&1 | tee $O/ab_cfg5.txt
