#!/bin/bash
# the x3 act's row order by (table path, window centre) (EVX_ACT_ROWPERM): its tests, the act
# microbenchmark in three row orders, then an A/B of the default bench
set -o pipefail
O=gpurun_out/rowperm; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_act_rowperm_gpu.py tests/test_draws_gpu.py \
  tests/test_trainer_gpu.py tests/test_qmlp_x3_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
for o in env centre shuffle; do timeout -k 10 120 python3 tools/act3_bench.py --table-frac 1.0 --order $o 2>&1 | tail -1 | sed "s/^/order $o: /"; done
for i in 1 2; do
  for s in 1 0; do
    EVX_ACT_ROWPERM=$s timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 \
      --other-steps 0 > $O/b_${s}_$i.json 2> $O/b_${s}_$i.err || { tail $O/b_${s}_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${s}_$i.json')); print('rowperm=$s', round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['env_step_kernel_ms'],3), round(d['learn_ms'],3))"
  done
done
