#!/bin/bash
# EVX_ORDER_INLINE A/B on the default bench (extras off) + step timeline of the inline run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in 0 1 0 1; do
  EVX_ORDER_INLINE=$v timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 \
     > $R/gpurun_out/inl.json 2> $R/gpurun_out/inl.err || { tail $R/gpurun_out/inl.err; exit 1; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/inl.json')); print('inline=$v value', round(d['value']/1e6,3), 'ms', round(d['ms_per_step'],3), 'env', round(d['env_step_kernel_ms'],3), 'learn', round(d['learn_ms'],3))"
done
EVX_ORDER_INLINE=1 bash $R/tools/gpu_steptrace.sh inl 26
