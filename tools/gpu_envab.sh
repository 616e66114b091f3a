#!/bin/bash
# env-only bench A/B over experiment builds (EVX_LIB): default then each libevacx_<tag>.so; extra args to bench.py
set -o pipefail
TAGS="$1"; shift
for tag in default $TAGS; do
  if [ "$tag" = default ]; then L=""; else L="EVX_LIB=$PWD/dqn-marl_amd/evacx/libevacx_$tag.so"; fi
  env $L timeout -k 10 300 python bench.py --mode env --no-cpu --steps 20 --warmup 3 "$@" > gpurun_out/envab_$tag.json 2> gpurun_out/envab_$tag.err || { tail -3 gpurun_out/envab_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/envab_$tag.json')); print('$tag', 'env-only %.3f M/s' % (d['value']/1e6), 'kernel %.3f ms' % d['env_step_kernel_ms'])"
done
