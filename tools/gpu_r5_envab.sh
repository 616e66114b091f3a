#!/bin/bash
# round 5: env_step occupancy A/B (EVX_LIB variants): default (3 waves/SIMD, GQ 2, LDS bitmaps),
# w4g1 (4 waves/SIMD cap, GQ 1), w4g1b (+ every grid's bitmaps in global scratch: 10 KB LDS per env),
# g1b (GQ 1, global bitmaps, 3 waves/SIMD); env-only at cfg3 (32768 envs, stationary mix)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5envab; rm -rf $OUT; mkdir -p $OUT
cd $R
for i in 1 2; do
  for v in default w4g1 w4g1b g1b; do
    L=""; [ $v != default ] && L="$R/dqn-marl_amd/evacx/libevacx_$v.so"
    EVX_LIB=$L timeout -k 10 300 python3 bench.py --mode env --steps 30 --warmup 3 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0 \
      > $OUT/e_${v}_$i.json 2> $OUT/e_${v}_$i.err || { tail -5 $OUT/e_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/e_${v}_$i.json')); print('$v', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'env %.4f' % d['env_step_kernel_ms'])"
  done
done
EVX_LIB=$R/dqn-marl_amd/evacx/libevacx_w4g1b.so timeout -k 10 300 python3 tools/stamp_probe.py --envs 32768 > $OUT/stamps_w4g1b.txt 2>&1 || { tail $OUT/stamps_w4g1b.txt; exit 1; }
head -4 $OUT/stamps_w4g1b.txt; grep "launch span" $OUT/stamps_w4g1b.txt
