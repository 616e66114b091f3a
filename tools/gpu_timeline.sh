#!/bin/bash
# Kernel timeline of the training step (lagged schedule) + the MLP microbenchmark.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tl
mkdir -p "$OUT"
timeout -k 10 200 python3 "$R/tools/qmlp_bench.py" > "$OUT/qmlp.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 20 --no-cpu --env-steps 0 --strict-steps 0 "$@" > "$OUT/bench.log" 2>&1 || exit 1
f=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/step_timeline.py" "$f" > "$OUT/timeline.txt"
cat "$OUT/qmlp.log" "$OUT/timeline.txt"
