#!/bin/bash
# Heavy-env cap / threshold sweep on the full training step (lagged), after the round-1 kernel changes
CMS=("256 -1" "128 -1" "384 -1" "256 400" "256 800" "192 -1" "256 -1"); [ -n "$SWEEP" ] && IFS=, read -ra CMS <<< "$SWEEP"
for cm in "${CMS[@]}"; do
  set -- $cm
  EVX_HEAVY_CAP=$1 EVX_HEAVY_MIN=$2 timeout -k 10 200 python bench.py --no-cpu --env-steps 0 --strict-steps 0 > gpurun_out/tht_$1_$2.json 2>/dev/null || exit 1
  echo "$1 $2 $(python -c "import json;print(json.load(open('gpurun_out/tht_$1_$2.json'))['value'])")"
done
