#!/bin/bash
# round 6 (session 2): heavy-env cap / threshold sweep on the headline training step (EVX_HEAVY_CAP / EVX_HEAVY_MIN)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2o; mkdir -p $O
for i in 1 2; do
  for cm in 176:0 128:0 224:0 256:0 176:400 176:800; do
    c=${cm%:*}; m=${cm#*:}
    if [ $m -gt 0 ]; then export EVX_HEAVY_MIN=$m; else unset EVX_HEAVY_MIN; fi
    EVX_HEAVY_CAP=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 \
      --start-steps 0 > /tmp/s.json 2> /tmp/s.err || { tail /tmp/s.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/s.json')); print('cap $c min $m', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'env %.4f' % d['env_step_kernel_ms'])" | tee -a $O/sweep_cfg3.txt
  done
done
