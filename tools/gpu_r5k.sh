#!/bin/bash
# round 5: cfg2 / cfg5 strict training-step timelines with idle gaps (one step between env launches)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5k; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C2="--grid 64 --people 569 --robots 8 --envs 4096"
C5="--replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304"
for c in ${CFGS:-2 5}; do
  eval CC=\$C$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t$c -o run --output-format csv -- python3 $R/bench.py --steps 12 --warmup 3 \
      --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 $CC > $OUT/trace_cfg$c.json 2> $OUT/trace_cfg$c.err || { tail $OUT/trace_cfg$c.err; exit 1; }
  python3 $R/tools/step_gaps.py $OUT/t$c > $OUT/step_gaps_cfg$c.txt 2>&1; tail -16 $OUT/step_gaps_cfg$c.txt
  rm -rf $OUT/t$c
done
