#!/bin/bash
# round 6 (session 2): qbwd3 with dZ2 staged for 16-B stores and 64-row blocks at B >= 16384: learn parity,
# learn kernel profile, cfg3 A/B (old, 128-row blocks + staging, 64-row blocks + staging)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2k; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_scale_gpu.py \
  tests/test_qmlp_x3_gpu.py tests/test_trainer_gpu.py tests/test_learner_golden_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
for v in libevacx_old.so libevacx_qb128.so libevacx.so; do
  EVX_LIB=$R/dqn-marl_amd/evacx/$v bash tools/gpu_prof.sh s2k/learn_$v -- python3 $R/tools/learn_bench.py 32768 10 table > $O/l_$v.txt 2>&1 || exit 1
  echo $v; python3 tools/kstat_csv.py $O/learn_$v/kernel_stats.csv 30 | grep -E "qbwd3|reduce2"
done
bash tools/gpu_abtrain.sh libevacx_old.so libevacx_qb128.so libevacx.so 2>&1 | tee $O/ab.txt
