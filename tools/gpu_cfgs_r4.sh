#!/bin/bash
# The other BASELINE configs as bench lines (cfg2, cfg5 = prioritized replay, cfg4 = conv Q-net) under gpurun_out/cfgs_<tag>
set -o pipefail
TAG=${1:-r4a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cfgs_$TAG; mkdir -p $OUT
cd "$R"
summ() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn', d['learn_ms'], 'frac %.3f' % d['roofline']['frac'])"; }
timeout -k 10 300 python3 bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 --env-steps 0 \
    > "$OUT/bench_cfg2.json" 2> "$OUT/bench_cfg2.err" || { tail -5 "$OUT/bench_cfg2.err"; exit 1; }
summ $OUT/bench_cfg2.json cfg2
timeout -k 10 400 python3 bench.py --no-cpu --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 --env-steps 0 \
    > "$OUT/bench_cfg5.json" 2> "$OUT/bench_cfg5.err" || { tail -5 "$OUT/bench_cfg5.err"; exit 1; }
summ $OUT/bench_cfg5.json cfg5
timeout -k 10 500 python3 bench.py --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 \
    --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 20 --other-steps 0 --start-steps 0 --batch 1024 \
    > "$OUT/bench_cfg4.json" 2> "$OUT/bench_cfg4.err" || { tail -5 "$OUT/bench_cfg4.err"; exit 1; }
summ $OUT/bench_cfg4.json cfg4
