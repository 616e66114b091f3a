#!/bin/bash
# kernel trace of the default training step (extras off) and the last two steps' timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/steptrace_${1:-a}; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value', d['value']/1e6, 'ms', d['ms_per_step'], 'env', d['env_step_kernel_ms'], 'learn', d['learn_ms'])"
python3 $R/tools/step_timeline.py $OUT/t ${2:-26}
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv ;
