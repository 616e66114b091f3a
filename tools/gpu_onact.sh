#!/bin/bash
# learner online forward through the fused act kernel (EVX_ONLINE_ACT): learn parity suites, then an A/B
set -o pipefail
O=gpurun_out/onact; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_scale_gpu.py::test_x3_learn_at_bench_batch \
  tests/test_split_learn_gpu.py tests/test_learner_golden_gpu.py tests/test_qmlp_x3_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  for s in 1 0; do
    EVX_ONLINE_ACT=$s timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 \
      --other-steps 0 > $O/b_${s}_$i.json 2> $O/b_${s}_$i.err || { tail $O/b_${s}_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${s}_$i.json')); print('online_act=$s', round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['env_step_kernel_ms'],3), round(d['learn_ms'],3), round(d['learn_alone_ms'],3))"
  done
done
