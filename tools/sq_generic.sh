#!/bin/bash
# One PMC pass of SQ issue/wait counters over any python command (kernel trace only).
#   tools/sq_generic.sh TAG python3 script.py args...   (run through gpurun from the repo root)
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
    -d "$OUT/sq" -o run --output-format csv -- "$@" > "$OUT/run.log" 2>&1
echo "profiles in $OUT"
