#!/bin/bash
# round 6: HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter per pass) of the act and the learn chain
# at cfg3's sizes (tools/act3_bench.py 524288 rows table path; tools/learn_bench.py 32768 table)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for w in "act:python3 $R/tools/act3_bench.py --table-frac 1.0" "learn:python3 $R/tools/learn_bench.py 32768 10 table"; do
  n=${w%%:*}; c=${w#*:}
  OUT=$R/gpurun_out/traf6_$n; rm -rf $OUT; mkdir -p $OUT
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fe -o run --output-format csv -- $c > $OUT/fe.log 2>&1 || { tail $OUT/fe.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/wr -o run --output-format csv -- $c > $OUT/wr.log 2>&1 || { tail $OUT/wr.log; exit 1; }
  python3 $R/tools/ktraffic.py $OUT/fe $OUT/wr 14 > $OUT/traffic.txt 2>&1; echo "== $n"; cat $OUT/traffic.txt
  rm -rf $OUT/fe $OUT/wr
done
