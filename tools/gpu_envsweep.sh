#!/bin/bash
# env parity suites, then the NWB sweep across env counts / configs
set -o pipefail
mkdir -p gpurun_out/envsweep
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py tests/test_layoutset_gpu.py -m gpu > gpurun_out/envsweep/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/envsweep/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_nwb2.sh
