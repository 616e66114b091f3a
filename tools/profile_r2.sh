#!/bin/bash
# Round-2 measurement on a GPU box (run through gpurun from the repo root):
#   bench.json           -- the driver's own command (bench.py --steps 20 --warmup 5), CPU baseline included
#   train_<phase>/       -- rocprofv3 --kernel-trace --stats of the same command (extras off, so the last
#                           launches of every kernel are the timed region)
#   fetch_/write_<phase> -- FETCH_SIZE and WRITE_SIZE of env_step_kernel, each in its own --pmc pass,
#                           counters collected only for env_step_kernel launches 1290.. (the timed region
#                           and the warm-up steps; the 1300-step preparation is not counted)
# for the stationary phase (the headline) and, trace only, the start phase. Summarise with
# tools/parse_prof_r2.py.
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
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/train_$PH" -o run --output-format csv -- \
      python3 "$R/bench.py" $X > "$OUT/train_$PH.log" 2>&1 || exit $?
  echo "trace $PH done"
  [ "$PH" = "start" ] && break
  for C in FETCH_SIZE WRITE_SIZE; do
    c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
    timeout -k 10 500 rocprofv3 --pmc $C --kernel-include-regex env_step_kernel --kernel-iteration-range "[1290-1400]" \
        -d "$OUT/${c}_$PH" -o run --output-format csv -- python3 "$R/bench.py" $X > "$OUT/${c}_$PH.log" 2>&1 || exit $?
    echo "$C $PH done"
  done
done
echo "profiles in $OUT"
