#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -x -v --timeout 200 --timeout-method thread -k "parts or split or order_ahead" > gpurun_out/t_split.log 2>&1 || { tail -30 gpurun_out/t_split.log; exit 1; }
tail -3 gpurun_out/t_split.log
timeout -k 10 300 python tools/split_probe.py > gpurun_out/split_probe.log 2>&1 || { tail -20 gpurun_out/split_probe.log; exit 1; }
cat gpurun_out/split_probe.log
