#!/bin/bash
# kernel trace of the default training step; the timeline of its last kernels (the learn-alone
# reading's 6 learns come last, the timed training steps before them)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/steptrace_r4; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 $R/tools/step_timeline.py $OUT/t 160 > $OUT/timeline.txt 2>&1 || true
rm -rf $OUT/t
grep -c . $OUT/timeline.txt
