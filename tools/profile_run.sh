#!/bin/bash
# Profile the bench on a GPU box (run through gpurun from the repo root):
#   1. kernel trace + stats of the full training step (train mode)
#   2. kernel trace + stats of env-only steps
#   3./4. FETCH_SIZE and WRITE_SIZE of env_step_kernel, each in its own pass
# Outputs under gpurun_out/prof_<tag>/; summarise with tools/parse_prof.py.
set -e
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 20 --no-cpu --env-steps 0 --strict-steps 0 > "$OUT/train.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/env" -o run --output-format csv -- \
    python3 "$R/bench.py" --mode env --steps 30 --no-cpu > "$OUT/env.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 "$R/bench.py" --mode env --steps 10 --no-cpu > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 "$R/bench.py" --mode env --steps 10 --no-cpu > "$OUT/write.log" 2>&1
echo "profiles in $OUT"
