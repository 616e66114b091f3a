#!/bin/bash
# In-box A/B of env_step builds (EVX_LIB): bench.py --mode env at cfg3, env_step_kernel_ms, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=$R/dqn-marl_amd/evacx
for i in 1 2; do
  for lib in "$@"; do
    EVX_LIB=$L/$lib timeout -k 10 200 python bench.py --mode env --steps 40 --warmup 5 --no-cpu --env-steps 0 \
      --other-steps 0 --start-steps 0 > /tmp/abenv.json 2> /tmp/abenv.err || { tail /tmp/abenv.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/abenv.json')); print('$lib', 'env %.4f ms' % d['env_step_kernel_ms'], 'value %.2f M' % (d['value']/1e6))"
  done
done
