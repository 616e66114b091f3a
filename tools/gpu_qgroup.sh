#!/bin/bash
# grouped independent nets (F3) parity suite
set -o pipefail
mkdir -p gpurun_out/qgroup
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_qgroup_gpu.py -m gpu > gpurun_out/qgroup/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/qgroup/pytest.log | head -40
exit $rc
