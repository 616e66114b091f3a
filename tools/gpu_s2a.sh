#!/bin/bash
# round 6 (session 2): rest-kernel probes, learn-forward parity, training-step A/B old vs new
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2a; mkdir -p $O
for v in r1 r2; do
  EVX_LIB=$R/dqn-marl_amd/evacx/libevacx_$v.so bash tools/gpu_prof.sh s2a/act_$v -- python3 $R/tools/act3_bench.py --table-frac 1.0 > $O/act_$v.txt 2>&1 || { tail $O/act_$v.txt; exit 1; }
  grep -E "rows|qact" $O/act_$v.txt
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_target_table_gpu.py \
  tests/test_bench_scale_gpu.py tests/test_trainer_gpu.py tests/test_learner_golden_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so 2>&1 | tee $O/ab.txt
