#!/bin/bash
# round 5: kernel timeline of one strict training step with the idle gaps between kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5gaps; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { tail $OUT/trace_bench.err; exit 1; }
python3 $R/tools/step_gaps.py $OUT/t > $OUT/step_gaps.txt 2>&1; tail -40 $OUT/step_gaps.txt
rm -rf $OUT/t
