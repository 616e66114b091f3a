#!/bin/bash
# round 5: env.step prefetch of env (slot + D)'s MT states / rmap / first in-play entries into L2 (libevacx_pf<D>.so)
# vs the default build: env parity at bench scale on pf256, then env-only and training-step lines alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5pf; rm -rf $OUT; mkdir -p $OUT
cd $R
EVX_LIB=$R/dqn-marl_amd/evacx/libevacx_pf256.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_env_gpu.py tests/test_order_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/tests.log | head -30; exit $rc; }
for i in 1 2; do
for tag in default pf128 pf256 pf512; do
  L=$R/dqn-marl_amd/evacx/libevacx.so; [ $tag != default ] && L=$R/dqn-marl_amd/evacx/libevacx_$tag.so
  EVX_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --steps 60 --warmup 10 --other-steps 0 --env-steps 100 --start-steps 0 \
      > $OUT/c3_${tag}_$i.json 2> $OUT/c3_${tag}_$i.err || { tail -5 $OUT/c3_${tag}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/c3_${tag}_$i.json'))
print('$tag', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'env %.4f' % d['env_step_kernel_ms'], 'env-only %.2f M' % (d['env_only_steps_per_s']/1e6))"
done; done
