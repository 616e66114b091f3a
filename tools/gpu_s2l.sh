#!/bin/bash
# round 6 (session 2): prioritized sampling two tree levels per load round: parity vs the oracle, cfg5 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_prio_gpu.py \
  tests/test_distributed_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
A="--robots 32 --envs 8192 --replay prioritized --replay-capacity 4194304"
bash tools/gpu_prof.sh s2l/cfg5 -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 $A > $O/cfg5.txt 2>&1 || { tail $O/cfg5.txt; exit 1; }
python3 tools/step_kstats.py $O/cfg5 20 | head -30
bash tools/gpu_abtrain.sh libevacx_old.so libevacx.so -- $A 2>&1 | tee $O/ab_cfg5.txt
