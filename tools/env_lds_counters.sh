#!/bin/bash
# LDS and issue counters of env_step_kernel on env-only bench steps (one PMC pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/envlds
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU \
    -d "$OUT/p" -o run --output-format csv -- python3 "$R/bench.py" --mode env --steps 10 --no-cpu > "$OUT/p.log" 2>&1 || exit 1
f=$(find "$OUT/p" -name "*counter_collection.csv" | head -1)
python3 "$R/tools/sq_summary.py" "$f" env_step_kernel
