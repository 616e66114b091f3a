#!/bin/bash
# x3 act table path + env order: numerics tests, trainer tests, bench (default workload), act microbench
set -o pipefail
mkdir -p gpurun_out/as
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_trainer_gpu.py tests/test_draws_gpu.py tests/test_qmlp_gpu.py tests/test_learner_golden_gpu.py > gpurun_out/as/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/as/bench.json 2> gpurun_out/as/bench.err
echo "bench rc=$?"
EVX_ACT_STATIC=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > gpurun_out/as/bench_nostatic.json 2> gpurun_out/as/bench_nostatic.err
echo "bench nostatic rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/as/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/as/trace.log 2>&1
echo "trace rc=$?"
