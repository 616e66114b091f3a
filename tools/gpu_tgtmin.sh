#!/bin/bash
# cfg2 (B 4096) and cfg5 (B 8192): the target forward through the fused act kernel (with its table)
# from B >= EVX_TGT_ACT_MIN: 32768 (the default) vs 2048
set -o pipefail
O=gpurun_out/tgtmin; mkdir -p $O
for i in 1 2; do
  for m in 32768 2048; do
    EVX_TGT_ACT_MIN=$m timeout -k 10 300 python bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 --env-steps 0 \
      --other-steps 0 --start-steps 0 --steps 30 > $O/c2_${m}_$i.json 2> $O/c2_${m}_$i.err || { tail -5 $O/c2_${m}_$i.err; exit 1; }
    EVX_TGT_ACT_MIN=$m timeout -k 10 300 python bench.py --no-cpu --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 \
      --env-steps 0 --other-steps 0 --start-steps 0 --steps 30 > $O/c5_${m}_$i.json 2> $O/c5_${m}_$i.err || { tail -5 $O/c5_${m}_$i.err; exit 1; }
    for c in c2 c5; do python -c "
import json; d=json.load(open('$O/${c}_${m}_$i.json')); print('$c min=$m', round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['env_step_kernel_ms'],3), round(d['learn_ms'],3), d['learn_alone_ms'])"; done
  done
done
