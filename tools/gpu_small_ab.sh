#!/bin/bash
# A/B of two small schedule knobs on the default bench (both measured as noise, 17.76-17.87 M env-steps/s): EVX_SIDE_PRIO (the order kernels' side
# stream at high priority) and EVX_STAT_TILE (the act table rebuild in 64 x 256 tiles; removed from
# csrc/qmlp.hip after this A/B)
set -o pipefail
O=gpurun_out/small_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_draws_gpu.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
EVX_STAT_TILE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_qmlp_x3_gpu.py >> $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
echo "tests ok"
for i in 1 2; do
  for v in "A" "B" "C"; do
    case $v in A) E="";; B) E="EVX_SIDE_PRIO=-1";; C) E="EVX_STAT_TILE=1";; esac
    env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 \
      --other-steps 0 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail $O/b_${v}_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_$i.json')); print('$v $E', round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['env_step_kernel_ms'],3), round(d['learn_ms'],3), round(d['learn_alone_ms'],3))"
  done
done
