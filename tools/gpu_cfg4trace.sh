#!/bin/bash
# kernel stats of the cfg4 training step (conv Q-net x3, 8192 envs of 256x256, learn batch 1024)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cfg4trace; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --no-cpu --grid 256 \
    --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 3 --age-steps 300 --stagger 300 --steps 6 \
    --env-steps 0 --other-steps 0 --start-steps 0 --batch 1024 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 $R/tools/step_timeline.py $OUT/t 80 > $OUT/timeline.txt 2>&1 || true
rm -rf $OUT/t
head -30 $OUT/kernel_stats.csv | cut -c1-200
