#!/bin/bash
# F4 device floor field: parity tests + throughput.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_floor_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_floor.log 2>&1 || { tail -40 gpurun_out/t_floor.log; exit 1; }
tail -3 gpurun_out/t_floor.log
timeout -k 10 200 python tools/floor_bench.py > gpurun_out/floor_bench.log 2>&1 || { tail -20 gpurun_out/floor_bench.log; exit 1; }
cat gpurun_out/floor_bench.log
