#!/bin/bash
# the learner's online fc1 tile at B = 32768 (EVX_FC1X3: 0 = 64 x 128 (default), 11 = 64 x 256, 13 = 128 x 256 of
# 8 waves): learn microbenchmark, then the default bench line
set -o pipefail
O=gpurun_out/fc1ab; mkdir -p $O
for v in 0 11 13; do
  EVX_FC1X3=$v timeout -k 10 200 python3 tools/learn_bench.py 32768 30 > $O/lb_$v.txt 2>&1 || { tail $O/lb_$v.txt; exit 1; }
  echo "fc1x3=$v $(grep learn $O/lb_$v.txt | tail -1)"
done
EVX_FC1X3=11 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_bench_scale_gpu.py::test_x3_learn_at_bench_batch" > $O/pt11.log 2>&1; echo "fc1x3=11 parity rc=$?"
EVX_FC1X3=13 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_bench_scale_gpu.py::test_x3_learn_at_bench_batch" > $O/pt13.log 2>&1; echo "fc1x3=13 parity rc=$?"
