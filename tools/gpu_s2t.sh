#!/bin/bash
# round 6 (session 2): workgroup sums (clip norm partials / norm) by wave butterfly: learn parity, cfg3 / cfg2 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2t; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_qmlp_x3_gpu.py \
  tests/test_qmlp_gpu.py tests/test_learner_golden_gpu.py tests/test_qgroup_gpu.py tests/test_trainer_gpu.py \
  tests/test_distributed_gpu.py tests/test_qnet_gpu.py tests/test_qmix_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu_prof.sh s2t/cfg3 -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $O/cfg3.txt 2>&1 || { tail $O/cfg3.txt; exit 1; }
python3 tools/step_kstats.py $O/cfg3 20 | grep -E "reduce2|adam"
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so 2>&1 | tee $O/ab_cfg3.txt
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- --grid 64 --people 569 --robots 8 --envs 4096 2>&1 | tee $O/ab_cfg2.txt
