#!/bin/bash
# learn chain kernel trace (tools/learn_bench.py) with the online forward through the fused act
# kernel and through qfc1 + qfc23 (EVX_ONLINE_ACT=1 / 0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
B=${1:-32768}
cd /tmp && export TMPDIR=/tmp
for s in 1 0; do
  OUT=$R/gpurun_out/learntrace_$s; mkdir -p $OUT
  EVX_ONLINE_ACT=$s timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/tools/learn_bench.py $B 20 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
  echo "online_act=$s: $(grep learn $OUT/trace.log | tail -1)"
  f=$(find $OUT/t -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in sorted(csv.DictReader(open('$f')), key=lambda r: -float(r['TotalDurationNs'])):
    print('  %8.1f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:80]))
"
done
