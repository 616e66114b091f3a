#!/bin/bash
# long 128x128 reference replay, stationary-mix parity at bench scale, draw restatements
set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_draws_gpu.py "tests/test_env_gpu.py::test_gpu_replays_reference_trajectory" tests/test_env_gpu.py::test_stationary_mix_matches_oracle_at_bench_scale > gpurun_out/r2c/pytest.log 2>&1
echo "pytest rc=$?"
