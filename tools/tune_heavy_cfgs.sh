#!/bin/bash
# Heavy-env cap across schedules / configs: strict cfg3, env-only cfg3, cfg2, cfg5 (prioritized)
B="timeout -k 10 200 python bench.py --no-cpu --env-steps 0 --strict-steps 0"
for cap in 256 176 160; do
  for c in "strict:--schedule strict" "env:--mode env" "cfg2:--grid 64 --people 569 --robots 8" \
           "cfg5:--envs 8192 --robots 32 --replay prioritized"; do
    n=${c%%:*}; a=${c#*:}
    EVX_HEAVY_CAP=$cap $B $a > gpurun_out/thc_${n}_$cap.json 2>/dev/null || exit 1
    echo "$n $cap $(python -c "import json;print(json.load(open('gpurun_out/thc_${n}_$cap.json'))['value'])")"
  done
done
