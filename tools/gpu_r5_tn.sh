#!/bin/bash
# round 5: backward GEMM experiments (timing only; libevacx_<tag>.so builds of qmlp.hip): learn_bench per-kernel
# times under rocprofv3 at B = 32768 and 4096
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5tn; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for B in ${BS:-32768 4096}; do
for tag in ${TAGS:-default base tn2 noload qzlate qznof}; do
  L=$R/dqn-marl_amd/evacx/libevacx.so; [ $tag != default ] && L=$R/dqn-marl_amd/evacx/libevacx_$tag.so
  EVX_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/tools/learn_bench.py $B 30 table > $OUT/lb.log 2>&1 || { tail $OUT/lb.log; exit 1; }
  f=$(find $OUT/t -name "*kernel_stats.csv" | head -1)
  echo "$tag B=$B $(grep -o 'learn B=.*' $OUT/lb.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if any(k in n for k in ('gemm_tn','bwd_mid','reduce2','qbwd3')):
        print('   %8.1f us x %4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], n[:60]))"
  rm -rf $OUT/t
done; done
