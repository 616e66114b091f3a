#!/bin/bash
# rocprofv3 kernel-trace stats of one command: gpu_prof.sh TAG -- cmd args...
# -> gpurun_out/<TAG>/kernel_stats.csv (+ the command's stdout / stderr)
set -o pipefail
TAG=$1; shift; [ "$1" = "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- "$@" > $OUT/out.txt 2> $OUT/err.txt \
  || { tail -5 $OUT/err.txt; exit 1; }
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/t -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/t
tail -2 $OUT/out.txt
python3 $R/tools/kstat_csv.py $OUT/kernel_stats.csv 12
