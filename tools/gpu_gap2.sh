#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gap2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python3 "$R/tools/gap_probe2.py" > "$OUT/log" 2>&1 || exit 1
f=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/gap_probe2_parse.py" "$f"
