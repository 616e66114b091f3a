#!/bin/bash
# x3 (f32-accurate) MLP kernels: numerics tests, reference-pinned learner tests, bench
set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_learner_golden_gpu.py tests/test_qmlp_gpu.py tests/test_qnet_gpu.py > gpurun_out/r2b/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r2b/bench_f32.json 2> gpurun_out/r2b/bench_f32.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --precision bf16 --env-steps 0 --start-steps 0 > gpurun_out/r2b/bench_bf16.json 2> gpurun_out/r2b/bench_bf16.err
echo "bench rc=$?"
