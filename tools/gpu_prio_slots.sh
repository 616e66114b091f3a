#!/bin/bash
# env.step wave-priority sweep (EVX_PRIO_SLOTS; 0 = off) on the env-only and training benches
set -o pipefail
mkdir -p gpurun_out
for ps in 0 1 256 768 1536; do
  EVX_PRIO_SLOTS=$ps timeout -k 10 300 python bench.py --no-cpu --mode env > gpurun_out/ps_env_$ps.json 2>/dev/null || exit 1
  EVX_PRIO_SLOTS=$ps timeout -k 10 300 python bench.py --no-cpu --env-steps 0 --strict-steps 0 > gpurun_out/ps_tr_$ps.json 2>/dev/null || exit 1
  python -c "import json;a=json.load(open('gpurun_out/ps_env_$ps.json'));b=json.load(open('gpurun_out/ps_tr_$ps.json'));print('pslots $ps env-mode kernel %.4f value %.3fM | train value %.3fM ms %.4f kernel %.4f' % (a['env_step_kernel_ms'], a['value']/1e6, b['value']/1e6, b['ms_per_step'], b['env_step_kernel_ms']))"
done
