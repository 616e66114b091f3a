#!/bin/bash
# round 5: cfg3 / cfg2 lines of the current build against libevacx_old.so (an earlier commit's kernels) on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5abc3; rm -rf $OUT; mkdir -p $OUT
cd $R
for i in 1 2; do
for tag in new old; do
  L=$R/dqn-marl_amd/evacx/libevacx.so; [ $tag = old ] && L=$R/dqn-marl_amd/evacx/libevacx_old.so
  EVX_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --steps 100 --warmup 10 --other-steps 0 --env-steps 0 --start-steps 0 \
      > $OUT/c3_${tag}_$i.json 2> $OUT/c3_${tag}_$i.err || { tail -5 $OUT/c3_${tag}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/c3_${tag}_$i.json'))
print('cfg3 $tag', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'env %.4f' % d['env_step_kernel_ms'], 'learn', round(d['learn_ms'],4))"
done; done
