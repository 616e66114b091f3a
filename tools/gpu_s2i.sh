#!/bin/bash
# round 6 (session 2): learn X copied from the table rows X: parity, A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2i; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_qmlp_x3_gpu.py \
  tests/test_target_table_gpu.py tests/test_bench_scale_gpu.py tests/test_trainer_gpu.py tests/test_qmlp_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu_prof.sh s2i/train -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $O/train.txt 2>&1 || { tail $O/train.txt; exit 1; }
python3 tools/kstat_csv.py $O/train/kernel_stats.csv 30 | grep -E "x_expand"
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so 2>&1 | tee $O/ab.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- --robots 32 --envs 8192 --replay prioritized --replay-capacity 4194304 2>&1 | tee $O/ab_cfg5.txt
