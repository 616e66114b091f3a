#!/bin/bash
# drop-in API tests (patrol, float actions, gauss_next, trajectories, agent init)
set -o pipefail
mkdir -p gpurun_out/r2e
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dropin_gpu.py > gpurun_out/r2e/pytest.log 2>&1
echo "pytest rc=$?"
