#!/bin/bash
# round 6 (session 2): the strict schedule's priority update on its own stream: prioritized parity /
# determinism tests, cfg5 A/B (the previous commit's trainer vs this one, same library)
# (the "old" trainer: tools/ab/trainer_old.py = `git show 2c4571f:dqn-marl_amd/evacx/trainer.py`, written before the run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2m; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_prio_gpu.py \
  tests/test_distributed_gpu.py tests/test_trainer_gpu.py tests/test_concurrency_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
A="--robots 32 --envs 8192 --replay prioritized --replay-capacity 4194304"
set -e; rm -rf /tmp/oldrepo && mkdir -p /tmp/oldrepo && cp -r $R/bench.py $R/dqn-marl_amd $R/profiles /tmp/oldrepo/ && \
  cp $R/tools/ab/trainer_old.py /tmp/oldrepo/dqn-marl_amd/evacx/trainer.py
for i in 1 2; do
  for v in old new; do
    D=$R; [ $v = old ] && D=/tmp/oldrepo
    timeout -k 10 300 python $D/bench.py --steps 30 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 $A > /tmp/b.json 2> /tmp/b.err || { tail /tmp/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/b.json')); print('$v', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'learn %.4f' % d['learn_ms'])" | tee -a $O/ab_cfg5.txt
  done
done
