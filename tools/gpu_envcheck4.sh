#!/bin/bash
# env parity suites, then env-only A/B (default build vs experiment builds) at cfg5 and cfg3 geometry
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_env_gpu.py tests/test_bench_scale_gpu.py tests/test_dropin_gpu.py tests/test_layoutset_gpu.py \
    tests/test_order_gpu.py > gpurun_out/envcheck.log 2>&1
rc=$?; tail -2 gpurun_out/envcheck.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/envcheck.log | head -20; exit $rc; }
bash tools/gpu_envab.sh "$1" --robots 32 --envs 8192 && bash tools/gpu_envab.sh "$1"
