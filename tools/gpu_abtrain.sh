#!/bin/bash
# In-box A/B of builds (EVX_LIB) on the headline training step (cfg3 strict, stationary mix), interleaved;
# extra bench.py arguments after "--"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=$R/dqn-marl_amd/evacx
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done; [ "$1" = "--" ] && shift
for i in 1 2; do
  for lib in "${libs[@]}"; do
    EVX_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 \
      --start-steps 0 "$@" > /tmp/abt.json 2> /tmp/abt.err || { tail /tmp/abt.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/abt.json')); print('$lib', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'env %.4f' % d['env_step_kernel_ms'], 'learn %.4f' % (d['learn_ms'] or 0))"
  done
done
