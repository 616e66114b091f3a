#!/bin/bash
# Memory-side counters of the x3 act (tools/act3_bench.py, 524288 rows, table fraction 1.0):
# L1 -> L2 read requests and L2 hits / misses per launch (two PMC passes + a kernel trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/actmem; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/tools/act3_bench.py --table-frac 1.0 --iters 5 --order ${1:-env}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- $CMD > $OUT/t.log 2>&1 || { tail $OUT/t.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $OUT/p1 -o run --output-format csv -- $CMD > $OUT/p1.log 2>&1 || { tail $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/p2 -o run --output-format csv -- $CMD > $OUT/p2.log 2>&1 || { tail $OUT/p2.log; exit 1; }
grep -h "us per act\|TF" $OUT/t.log | tail -3
python3 - <<PY
import csv, glob, collections
for p in ("p1", "p2"):
    f = glob.glob("$OUT/%s/**/*counter_collection.csv" % p, recursive=True)[0]
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "qact3h" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, x in v.items():
        print(k, "per launch (last 3 mean): %.4g" % (sum(x[-3:]) / len(x[-3:])))
PY
