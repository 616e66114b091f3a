#!/bin/bash
# round 6 (session 2): split-K act table parity + the learn / act tests that read the table, table
# kernel timing in the training step, training-step A/B old vs new
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_qmlp_x3_gpu.py \
  tests/test_target_table_gpu.py tests/test_qmlp_gpu.py tests/test_trainer_gpu.py tests/test_bench_scale_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu_prof.sh s2c/train -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $O/train.txt 2>&1 || { tail $O/train.txt; exit 1; }
cat $O/train.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so 2>&1 | tee $O/ab.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- --grid 64 --people 569 --robots 8 --envs 4096 2>&1 | tee $O/ab_cfg2.txt
