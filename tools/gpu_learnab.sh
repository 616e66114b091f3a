#!/bin/bash
# learn-path parity (target / online tables, x3 learner, trainer), then the training step A/B:
# default build vs libevacx_<tag>.so (bench.py, strict schedule, learn_ms from its events)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_target_table_gpu.py tests/test_qmlp_x3_gpu.py tests/test_trainer_gpu.py tests/test_bench_scale_gpu.py > gpurun_out/learncheck.log 2>&1
rc=$?; tail -2 gpurun_out/learncheck.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/learncheck.log | head -30; exit $rc; }
for tag in default $1; do
  if [ "$tag" = default ]; then L=""; else L="EVX_LIB=$PWD/dqn-marl_amd/evacx/libevacx_$tag.so"; fi
  env $L timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 --other-steps 0 --env-steps 0 --start-steps 0 \
      > gpurun_out/learnab_$tag.json 2> gpurun_out/learnab_$tag.err || { tail -3 gpurun_out/learnab_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/learnab_$tag.json')); print('$tag', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn %.3f alone %.3f' % (d['learn_ms'], d['learn_alone_ms']))"
done
