#!/bin/bash
# round 5: env_step prefetch depth / occupancy A/B (EVX_LIB variants): GQ person groups in flight,
# waves per SIMD by VGPRs -- g4w2 (GQ 4, 2 waves/SIMD), g3w2 (GQ 3, 2), g1w3 (GQ 1, 3); env-only
# at cfg4 (256x256, 8192 envs) and cfg3 (128x128, 32768 envs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5envab2; rm -rf $OUT; mkdir -p $OUT
cd $R
C4="--grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --age-steps 300 --stagger 300"
for i in 1 2; do
  for v in default g4w2 g3w2 g1w3; do
    L=""; [ $v != default ] && L="$R/dqn-marl_amd/evacx/libevacx_$v.so"
    EVX_LIB=$L timeout -k 10 300 python3 bench.py --mode env --steps 10 --warmup 2 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0 $C4 \
      > $OUT/c4_${v}_$i.json 2> $OUT/c4_${v}_$i.err || { tail -5 $OUT/c4_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4_${v}_$i.json')); print('cfg4 $v', 'value %.4f M' % (d['value']/1e6), 'env %.4f' % d['env_step_kernel_ms'])"
  done
  for v in default g1w3 g3w2; do
    L=""; [ $v != default ] && L="$R/dqn-marl_amd/evacx/libevacx_$v.so"
    EVX_LIB=$L timeout -k 10 300 python3 bench.py --mode env --steps 30 --warmup 3 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0 \
      > $OUT/c3_${v}_$i.json 2> $OUT/c3_${v}_$i.err || { tail -5 $OUT/c3_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_${v}_$i.json')); print('cfg3 $v', 'value %.3f M' % (d['value']/1e6), 'env %.4f' % d['env_step_kernel_ms'])"
  done
done
