#!/bin/bash
# conv microbenchmark + one PMC pass of LDS / MFMA counters over it
set -o pipefail
O=gpurun_out/convb; mkdir -p $O
timeout -k 10 120 python tools/conv_bench.py > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
cat $O/bench.txt
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY \
    -d $R/$O/pmc -o run --output-format csv -- python3 $R/tools/conv_bench.py > $R/$O/pmc.log 2>&1 || { tail $R/$O/pmc.log; exit 1; }
cd $R
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/convb/pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
