#!/bin/bash
# round 5: Adam with ADAM_PT parameters per thread (default build: 4; _apt1: the previous one; _apt8) and the env's
# one-wave path at cfg2 (_nwb16): learner parity on the default build, then cfg2 / cfg3 lines alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5ab3; rm -rf $OUT; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_qmlp_x3_gpu.py tests/test_learner_golden_gpu.py \
  tests/test_trainer_gpu.py tests/test_qgroup_gpu.py tests/test_target_table_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/tests.log | head -30; exit $rc; }
summ() { python3 -c "
import json; d=json.load(open('$1'))
print('$2', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'env %.4f' % d['env_step_kernel_ms'], 'learn', d.get('learn_ms'), 'alone', d.get('learn_alone_ms'))"; }
for i in 1 2; do
for tag in default apt1 apt8 nwb16; do
  L=$R/dqn-marl_amd/evacx/libevacx.so; [ $tag != default ] && L=$R/dqn-marl_amd/evacx/libevacx_$tag.so
  EVX_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 --steps 300 --warmup 20 --other-steps 0 \
      --env-steps 0 --start-steps 0 > $OUT/c2_${tag}_$i.json 2> $OUT/c2_${tag}_$i.err || { tail -5 $OUT/c2_${tag}_$i.err; exit 1; }
  summ $OUT/c2_${tag}_$i.json "cfg2 $tag"
  if [ $tag != nwb16 ]; then
  EVX_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --steps 100 --warmup 10 --other-steps 0 --env-steps 0 --start-steps 0 \
      > $OUT/c3_${tag}_$i.json 2> $OUT/c3_${tag}_$i.err || { tail -5 $OUT/c3_${tag}_$i.err; exit 1; }
  summ $OUT/c3_${tag}_$i.json "cfg3 $tag"
  fi
done; done
