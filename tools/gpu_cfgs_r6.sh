#!/bin/bash
# round-6 evidence: the bench lines of cfg2 / cfg5 / cfg4 (BASELINE.json's other single-GPU configs)
# usage: tools/gpu_cfgs_r6.sh TAG
set -o pipefail
TAG=${1:-final_r6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
B="timeout -k 10 600 python3 bench.py --steps 20 --warmup 5"
$B --grid 64 --people 569 --robots 8 --envs 4096 > $OUT/bench_cfg2.json 2> $OUT/cfg2.err || { tail $OUT/cfg2.err; exit 1; }
$B --robots 32 --envs 8192 --replay prioritized --replay-capacity 4194304 > $OUT/bench_cfg5.json 2> $OUT/cfg5.err || { tail $OUT/cfg5.err; exit 1; }
$B --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --age-steps 300 --stagger 300 --batch 1024 > $OUT/bench_cfg4.json 2> $OUT/cfg4.err || { tail $OUT/cfg4.err; exit 1; }
for c in cfg2 cfg5 cfg4; do python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); r=d['roofline']; print('$c', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn %.3f' % d['learn_ms'], 'bound', r['bound'], 'frac %.3f' % r['frac'])"; done
