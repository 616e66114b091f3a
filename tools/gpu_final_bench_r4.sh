#!/bin/bash
# round-4 bench evidence: the driver's default line, its kernel trace / stats, the other configs' lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final_r4; mkdir -p $OUT
cd $R
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('cfg3', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn %.3f alone %.3f' % (d['learn_ms'], d['learn_alone_ms']), 'frac %.3f' % d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { tail -5 $OUT/trace_bench.err; exit 1; }
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 $R/tools/step_timeline.py $OUT/t 40 > $OUT/timeline.txt 2>&1 || true
rm -rf $OUT/t
cd $R
bash tools/gpu_cfgs_r4.sh final_r4
