#!/bin/bash
# A/B of the split learn step (EVX_SPLIT_LEARN) on one box, alternating
set -o pipefail
O=gpurun_out/ab_split; mkdir -p $O
for i in 1 2; do
  for s in 1 0; do
    EVX_SPLIT_LEARN=$([ $s = 0 ] && echo 0 || echo 1) timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 \
      --other-steps 0 > $O/b_${s}_$i.json 2> $O/b_${s}_$i.err || { tail $O/b_${s}_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${s}_$i.json')); print('split=$s', round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['env_step_kernel_ms'],3), round(d['learn_ms'],3))"
  done
done
