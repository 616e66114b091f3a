#!/bin/bash
# SQ issue/wait breakdown of env_step_kernel (one PMC pass, kernel trace only).
# Run through gpurun from the repo root; summarise with tools/parse_prof.py --sq.
set -e
TAG=${1:-sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU \
    -d "$OUT/sq" -o run --output-format csv -- \
    python3 "$R/bench.py" --mode env --steps 10 --no-cpu > "$OUT/sq.log" 2>&1
echo "profiles in $OUT"
