#!/bin/bash
# fused learner chain + parallel reward leaves: numerics tests, env parity, trainer tests, bench
set -o pipefail
mkdir -p gpurun_out/r2i
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_learner_golden_gpu.py tests/test_qmlp_gpu.py tests/test_trainer_gpu.py tests/test_distributed_gpu.py tests/test_prio_gpu.py tests/test_qnet_gpu.py > gpurun_out/r2i/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r2i/bench.json 2> gpurun_out/r2i/bench.err
echo "bench rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2i/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r2i/trace.log 2>&1
echo "trace rc=$?"
