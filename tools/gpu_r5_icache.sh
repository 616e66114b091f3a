#!/bin/bash
# round 5: instruction-cache counters of env_step_kernel (bench --mode env, cfg3 stationary mix)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5ic; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
( while sleep 20; do date >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -i -E "ICACHE|IFETCH|INST_LEVEL|SQC_TC" $OUT/avail.txt > $OUT/avail_ic.txt || true
CMD="python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0 --age-steps 250 --stagger 250"
timeout -s KILL 420 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d $OUT/ic -o run --output-format csv -- $CMD > $OUT/ic.log 2>&1 || { tail $OUT/ic.log; exit 1; }
python3 - $OUT/ic > $OUT/icache.txt <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:60]
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "env_step" in k or "orders" in k:
        print(k, {c: sum(v[-5:]) / len(v[-5:]) for c, v in d.items()})
PY
cat $OUT/icache.txt; rm -rf $OUT/ic
