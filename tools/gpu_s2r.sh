#!/bin/bash
# round 6 (session 2): env_step load phase in two dependent rounds of loads (header-independent reads
# issued before the list header's test): env parity, then cfg3 / cfg2 / cfg4 A/B against the previous build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2r; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_bench_scale_gpu.py tests/test_layoutset_gpu.py tests/test_order_gpu.py tests/test_dropin_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so 2>&1 | tee $O/ab_cfg3.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- --grid 64 --people 569 --robots 8 --envs 4096 2>&1 | tee $O/ab_cfg2.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --age-steps 300 --stagger 300 --batch 1024 2>&1 | tee $O/ab_cfg4.txt
