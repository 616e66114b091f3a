#!/bin/bash
# kernel-trace stats of the cfg4 bench (conv Q-net, 256x256, P 9102, 8192 envs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cfg4prof
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/t" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 3 --age-steps 300 --stagger 300 --steps 5 --env-steps 0 --other-steps 0 --start-steps 0 --batch 1024 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
f=$(find "$OUT/t" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
