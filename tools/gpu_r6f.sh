#!/bin/bash
# round 6: counter records of cfg2 / cfg5 / cfg4 (env_step: SQ + GRBM + PMC bytes), then every config's bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r6f
bash tools/gpu_r6_counters.sh cfg2 cfg5 cfg4 > gpurun_out/r6f/cnt.log 2>&1 || { tail -20 gpurun_out/r6f/cnt.log; exit 1; }
cp gpurun_out/r6cnt/env_counters_stationary_cfg*.json profiles/r6/
B="timeout -k 10 600 python3 bench.py --steps 20 --warmup 5"
$B --grid 64 --people 569 --robots 8 --envs 4096 > gpurun_out/r6f/bench_cfg2.json 2> gpurun_out/r6f/cfg2.err || { tail gpurun_out/r6f/cfg2.err; exit 1; }
$B --robots 32 --envs 8192 --replay prioritized --replay-capacity 4194304 > gpurun_out/r6f/bench_cfg5.json 2> gpurun_out/r6f/cfg5.err || { tail gpurun_out/r6f/cfg5.err; exit 1; }
$B --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --age-steps 300 --stagger 300 --batch 1024 > gpurun_out/r6f/bench_cfg4.json 2> gpurun_out/r6f/cfg4.err || { tail gpurun_out/r6f/cfg4.err; exit 1; }
for c in cfg2 cfg5 cfg4; do python3 -c "import json; d=json.load(open('gpurun_out/r6f/bench_$c.json')); r=d['roofline']; print('$c', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'bound', r['bound'], 'frac %.3f' % r['frac'], 'hbm traffic frac', d['roofline_hbm']['frac_traffic'])"; done
