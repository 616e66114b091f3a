#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2g
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dropin_gpu.py > gpurun_out/r2g/pytest.log 2>&1
echo "pytest rc=$?"
