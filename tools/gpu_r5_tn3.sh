#!/bin/bash
# round 5: the k-major x3 weight-gradient kernel (tn3_kernel: conv dW, fc dW) -- conv / gemm parity, cfg4 learn
# parity, then cfg4 lines against the previous commit's qnet (libevacx_old.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5tn3; rm -rf $OUT; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_qnet_gpu.py tests/test_env_gpu.py tests/test_qmix_golden_gpu.py tests/test_qgroup_gpu.py tests/test_dropin_gpu.py tests/test_layoutset_gpu.py \
  tests/test_bench_scale_gpu.py -k "conv or gemm or learn or qmix or dropin or group or obs or expand or layout" > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/tests.log | head -30; exit $rc; }
C4="--grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 0 --other-steps 0 --start-steps 0 --batch 1024 --no-cpu"
for i in 1 2; do
for tag in new old; do
  L=$R/dqn-marl_amd/evacx/libevacx.so; [ $tag = old ] && L=$R/dqn-marl_amd/evacx/libevacx_old.so
  EVX_LIB=$L timeout -k 10 400 python3 bench.py $C4 > $OUT/c4_${tag}_$i.json 2> $OUT/c4_${tag}_$i.err || { tail -5 $OUT/c4_${tag}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/c4_${tag}_$i.json'))
print('cfg4 $tag', 'value %.4f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn', d.get('learn_ms'), 'alone', d.get('learn_alone_ms'))"
done; done
