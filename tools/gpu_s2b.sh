#!/bin/bash
# round 6 (session 2): act workspace parity, act profile, training-step A/B old vs new
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_qmlp_x3_gpu.py \
  tests/test_trainer_gpu.py tests/test_concurrency_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu_prof.sh s2b/act -- python3 $R/tools/act3_bench.py --table-frac 1.0 > $O/act.txt 2>&1 || { tail $O/act.txt; exit 1; }
grep -E "rows|qact" $O/act.txt
bash tools/gpu_prof.sh s2b/act85 -- python3 $R/tools/act3_bench.py --table-frac 0.85 > $O/act85.txt 2>&1 || { tail $O/act85.txt; exit 1; }
grep -E "rows|qact" $O/act85.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so 2>&1 | tee $O/ab.txt
