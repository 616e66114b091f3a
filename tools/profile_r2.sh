#!/bin/bash
# Round-2 measurement on a GPU box (run through gpurun from the repo root):
#   bench.json          -- the driver's own command (bench.py --steps 20 --warmup 5), CPU baseline included
#   train_<phase>/      -- rocprofv3 --kernel-trace --stats of the same command (extras off, so the last
#                          launches of every kernel are the timed region)
#   fetch_/write_<phase>-- FETCH_SIZE and WRITE_SIZE of env_step_kernel, each in its own --pmc pass
# for the stationary phase (the headline) and the start phase. Summarise with tools/parse_prof_r2.py.
set -o pipefail
TAG=${1:-r2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 "$R/bench.py" --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
echo "bench done"
for PH in stationary start; do
  X="--steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 --phase $PH"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train_$PH" -o run --output-format csv -- \
      python3 "$R/bench.py" $X > "$OUT/train_$PH.log" 2>&1 || exit $?
  echo "trace $PH done"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch_$PH" -o run --output-format csv -- \
      python3 "$R/bench.py" $X > "$OUT/fetch_$PH.log" 2>&1 || exit $?
  echo "fetch $PH done"
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write_$PH" -o run --output-format csv -- \
      python3 "$R/bench.py" $X > "$OUT/write_$PH.log" 2>&1 || exit $?
  echo "write $PH done"
done
echo "profiles in $OUT"
