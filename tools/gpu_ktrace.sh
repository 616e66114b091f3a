#!/bin/bash
# kernel trace + per-kernel means of one command: tools/gpu_ktrace.sh NAME cmd...  (env passes through)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
OUT=$R/gpurun_out/kt_$N; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- "$@" > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
grep -E "us per|ms" $OUT/trace.log | tail -3
python3 $R/tools/kstats.py $OUT 3 > $OUT/kstats.txt && head -${KT_TOP:-14} $OUT/kstats.txt
