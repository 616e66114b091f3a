#!/bin/bash
# the learner's target forward from the target net's act table (EVX_TGT_TABLE): parity, then an A/B
set -o pipefail
O=gpurun_out/tgttab; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_target_table_gpu.py \
  tests/test_trainer_gpu.py tests/test_draws_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  for s in 1 0; do
    EVX_TGT_TABLE=$s timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 \
      --other-steps 0 > $O/b_${s}_$i.json 2> $O/b_${s}_$i.err || { tail $O/b_${s}_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${s}_$i.json')); print('tgt_table=$s', round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['env_step_kernel_ms'],3), round(d['learn_ms'],3), round(d['learn_alone_ms'],3))"
  done
done
