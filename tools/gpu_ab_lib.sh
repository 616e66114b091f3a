#!/bin/bash
# A/B of an experiment build (dqn-marl_amd/evacx/libevacx_old.so = the previous commit's kernels) against
# the current libevacx.so on one box: env parity suites on the current build, then alternating bench lines
set -o pipefail
O=gpurun_out/ab_lib; mkdir -p $O
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_env_gpu.py tests/test_bench_scale_gpu.py \
  tests/test_dropin_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  for v in new old; do
    L=""; [ $v = old ] && L="$R/dqn-marl_amd/evacx/libevacx_old.so"
    EVX_LIB=$L timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --env-steps 100 --start-steps 0 \
      --other-steps 0 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail $O/b_${v}_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_$i.json')); print('$v', round(d['value']/1e6,3), round(d['ms_per_step'],3), 'env', round(d['env_step_kernel_ms'],4), 'env-only', round(d['env_only_steps_per_s']/1e6,3))"
  done
done
