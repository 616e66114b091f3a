#!/bin/bash
# round 5: headline + cfg2 lines (no cpu baseline) with the timed region free of event records
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5b2; rm -rf $OUT; mkdir -p $OUT
cd $R
summ() { python3 -c "
import json; d=json.load(open('$1'))
print('$2', 'value %.3f M' % (d['value']/1e6), 'ms %.4f' % d['ms_per_step'], 'env %.4f' % d['env_step_kernel_ms'], 'learn', d.get('learn_ms'), 'frac %.3f' % d['roofline']['frac'])"; }
for i in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu --steps 100 --warmup 10 --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/c3_$i.json 2> $OUT/c3_$i.err || { tail -5 $OUT/c3_$i.err; exit 1; }
summ $OUT/c3_$i.json cfg3
timeout -k 10 300 python3 bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 --steps 300 --warmup 20 --other-steps 0 --env-steps 0 --start-steps 0 \
    > $OUT/c2_$i.json 2> $OUT/c2_$i.err || { tail -5 $OUT/c2_$i.err; exit 1; }
summ $OUT/c2_$i.json cfg2
done
