#!/bin/bash
# big-grid env parity (cfg4 geometry), then env-only A/B at cfg4 (default build vs libevacx_<tag>.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_bench_scale_gpu.py::test_cfg4_env_at_bench_scale tests/test_env_gpu.py tests/test_sort_gpu.py > gpurun_out/cfg4check.log 2>&1
rc=$?; tail -2 gpurun_out/cfg4check.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/cfg4check.log | head -20; exit $rc; }
bash tools/gpu_envab.sh "$1" --grid 256 --people 9102 --robots 1 --envs 8192 --age-steps 300 --stagger 300 --steps 10 --warmup 3
