#!/bin/bash
# round 5: small-batch forward tilings (libevacx_wide.so: forward2's fc1 in 64 x 256 tiles below 256
# workgroups; libevacx_narrow.so: the act-table rebuild in 64 x 64 tiles of 2 waves below 256 workgroups):
# parity on each, then cfg2 bench lines alternating with the default build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5small; rm -rf $OUT; mkdir -p $OUT
cd $R
for tag in ${VTAGS:-wide narrow}; do
  EVX_LIB=$R/dqn-marl_amd/evacx/libevacx_$tag.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_target_table_gpu.py tests/test_qmlp_x3_gpu.py tests/test_learner_golden_gpu.py tests/test_trainer_gpu.py tests/test_qmlp_gpu.py tests/test_bench_scale_gpu.py > $OUT/tests_$tag.log 2>&1
  rc=$?; echo "$tag: $(tail -1 $OUT/tests_$tag.log)"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/tests_$tag.log | head -30; exit $rc; }
done
summ() { python3 -c "
import json; d=json.load(open('$1'))
print('$2', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'env %.4f' % d['env_step_kernel_ms'], 'learn', d.get('learn_ms'), 'alone', d.get('learn_alone_ms'))"; }
for i in 1 2; do
for tag in default ${VTAGS:-wide narrow}; do
  L=$R/dqn-marl_amd/evacx/libevacx.so; [ $tag != default ] && L=$R/dqn-marl_amd/evacx/libevacx_$tag.so
  EVX_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 --steps 300 --warmup 20 --other-steps 0 \
      --env-steps 0 --start-steps 0 > $OUT/c2_${tag}_$i.json 2> $OUT/c2_${tag}_$i.err || { tail -5 $OUT/c2_${tag}_$i.err; exit 1; }
  summ $OUT/c2_${tag}_$i.json $tag
done; done
