#!/bin/bash
# kernel-trace stats of the headline bench (stationary phase, extras off)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_head; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/t" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > "$OUT/run.log" 2>&1 || { tail "$OUT/run.log"; exit 1; }
f=$(find "$OUT/t" -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
per = collections.defaultdict(list)
for r in rows:
    per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1][-19:])):
    t = v[-19:]
    print(f"{sum(t)/len(t):9.1f} us x{len(v):5d}  {k[:90]}")
PY
