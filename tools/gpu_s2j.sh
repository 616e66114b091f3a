#!/bin/bash
# round 6 (session 2): dZ1 tiles of 2 column tiles per wave: learn parity, A/B cfg3 / cfg5 / cfg2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2j; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_scale_gpu.py \
  tests/test_qmlp_x3_gpu.py tests/test_qmlp_gpu.py tests/test_trainer_gpu.py tests/test_learner_golden_gpu.py \
  tests/test_qgroup_gpu.py tests/test_distributed_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu_prof.sh s2j/learn -- python3 $R/tools/learn_bench.py 32768 10 table > $O/learn.txt 2>&1 || { tail $O/learn.txt; exit 1; }
python3 tools/kstat_csv.py $O/learn/kernel_stats.csv 30 | grep -E "bwd_mid"
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so 2>&1 | tee $O/ab.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- --grid 64 --people 569 --robots 8 --envs 4096 2>&1 | tee $O/ab_cfg2.txt
