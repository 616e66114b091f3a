#!/bin/bash
# kernel trace of the learn chain at cfg2's batch (B = 4096, tools/learn_bench.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/learn4k; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python3 $R/tools/learn_bench.py 4096 20 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
grep learn $OUT/trace.log | tail -1
f=$(find $OUT/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# the last learn step: from the last replay/forward kernel group
idx = [i for i, r in enumerate(rows) if "adam_pack3" in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 2
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print("%8.1f %8.1f %6.1f  %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r["Kernel_Name"][:70]))
PY
rm -rf $OUT/t
