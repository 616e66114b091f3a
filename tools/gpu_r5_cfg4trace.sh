#!/bin/bash
# round 5: cfg4 training-step kernel timeline (rocprofv3 kernel trace, the last learn's kernels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5c4t; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C4="--grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 3 --age-steps 300 --stagger 300 --steps 4 --env-steps 0 --other-steps 0 --start-steps 0 --batch 1024 --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py $C4 > $OUT/trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python3 $R/tools/step_timeline.py $OUT/t 75 > $OUT/timeline_cfg4.txt 2>&1 || true
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_cfg4.csv \;
rm -rf $OUT/t
