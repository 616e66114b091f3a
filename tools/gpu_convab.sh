#!/bin/bash
# conv Q-net parity suites, then the cfg4 training step A/B (default build vs libevacx_<tag>.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_qnet_gpu.py tests/test_gemm_epilogue_gpu.py tests/test_learner_golden_gpu.py \
    "tests/test_bench_scale_gpu.py::test_conv_x3_learn_at_cfg4_batch" tests/test_qmix_gpu.py > gpurun_out/convcheck.log 2>&1
rc=$?; tail -2 gpurun_out/convcheck.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/convcheck.log | head -30; exit $rc; }
for tag in default $1; do
  if [ "$tag" = default ]; then L=""; else L="EVX_LIB=$PWD/dqn-marl_amd/evacx/libevacx_$tag.so"; fi
  env $L timeout -k 10 500 python3 bench.py --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 \
      --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 0 --other-steps 0 --start-steps 0 --batch 1024 \
      > gpurun_out/convab_$tag.json 2> gpurun_out/convab_$tag.err || { tail -5 gpurun_out/convab_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/convab_$tag.json')); print('cfg4 $tag', 'value %.4f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn %.3f' % d['learn_ms'])"
done
