#!/bin/bash
# the act row order with the order kernels inline on the main stream (EVX_ORDER_INLINE=1) vs the defaults
set -o pipefail
O=gpurun_out/rp2; mkdir -p $O
for i in 1 2; do
  for v in A B C; do
    case $v in A) E="EVX_ACT_ROWPERM=0";; B) E="EVX_ACT_ROWPERM=1 EVX_ORDER_INLINE=1";; C) E="EVX_ACT_ROWPERM=0 EVX_ORDER_INLINE=1";; esac
    env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 \
      --other-steps 0 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail $O/b_${v}_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_$i.json')); print('$v $E', round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['env_step_kernel_ms'],3), round(d['learn_ms'],3))"
  done
done
