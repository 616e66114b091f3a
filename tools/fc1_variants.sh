#!/bin/bash
# fc1 tile variants (EVX_FC1_NWV) on the MLP microbenchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_qmlp_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/t_q.log 2>&1 || { tail -30 gpurun_out/t_q.log; exit 1; }
tail -1 gpurun_out/t_q.log
for v in 8 4; do
  echo "nwv $v"
  EVX_FC1_NWV=$v timeout -k 10 120 python tools/qmlp_bench.py 2>&1 | grep -E "fc1 only|act"
done
