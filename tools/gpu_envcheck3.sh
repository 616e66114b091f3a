#!/bin/bash
# env kernel change: the env parity suites, then the env-only rate and the phase stamps at 32768 envs
set -o pipefail
O=gpurun_out/envcheck3_${1:-a}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_env_gpu.py tests/test_bench_scale_gpu.py tests/test_dropin_gpu.py tests/test_layoutset_gpu.py -k "not learn" > $O/env.log 2>&1 || { grep -E "Error|assert|FAIL" $O/env.log | head -20; tail -5 $O/env.log; exit 1; }
tail -1 $O/env.log
timeout -k 10 300 python tools/stamp_probe.py --envs 32768 > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
grep -v Warn $O/stamps.txt | head -12
timeout -k 10 400 python bench.py --mode env --steps 30 --no-cpu > $O/benv.json 2> $O/benv.err || { tail $O/benv.err; exit 1; }
python -c "import json; d=json.load(open('$O/benv.json')); print('env-only', d['value'], 'kernel ms', d['env_step_kernel_ms'], 'frac', d['roofline']['frac'])"
