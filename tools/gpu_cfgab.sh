#!/bin/bash
# cfg2 / cfg5 training-step A/B: default build vs libevacx_<tag>.so
set -o pipefail
mkdir -p gpurun_out
for tag in default $1; do
  if [ "$tag" = default ]; then L=""; else L="EVX_LIB=$PWD/dqn-marl_amd/evacx/libevacx_$tag.so"; fi
  env $L timeout -k 10 300 python3 bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 --env-steps 0 --other-steps 0 --start-steps 0 \
      > gpurun_out/cfgab2_$tag.json 2> gpurun_out/cfgab2_$tag.err || { tail -5 gpurun_out/cfgab2_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cfgab2_$tag.json')); print('cfg2 $tag', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn %.3f alone %.3f' % (d['learn_ms'], d['learn_alone_ms']))"
  env $L timeout -k 10 400 python3 bench.py --no-cpu --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 --env-steps 0 --other-steps 0 --start-steps 0 \
      > gpurun_out/cfgab5_$tag.json 2> gpurun_out/cfgab5_$tag.err || { tail -5 gpurun_out/cfgab5_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cfgab5_$tag.json')); print('cfg5 $tag', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn %.3f alone %.3f' % (d['learn_ms'], d['learn_alone_ms']))"
done
