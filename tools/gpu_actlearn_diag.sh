#!/bin/bash
# act phase stamps (libevacx_actst.so, -DEVX_ACT_STAMPS) + learn chain kernel stats at B = 32768
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ald; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 python3 $R/tools/act_stamps.py 1.0 > $OUT/act_stamps.txt 2>&1 || { tail $OUT/act_stamps.txt; exit 1; }
grep -v Warning $OUT/act_stamps.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/tools/learn_bench.py 32768 20 > $OUT/learn.log 2>&1 || { tail $OUT/learn.log; exit 1; }
python3 $R/tools/kstats.py $OUT 1.0 > $OUT/learn_kstats.txt; cat $OUT/learn_kstats.txt; tail -3 $OUT/learn.log
rm -rf $OUT/t
