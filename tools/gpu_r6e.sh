#!/bin/bash
# env micro-opts: parity at bench scale, env A/B vs HEAD, act A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py tests/test_dropin_gpu.py 2>&1 | tail -2 || exit 1
bash tools/gpu_abenv.sh libevacx_head.so libevacx.so || exit 1
bash tools/gpu_abact.sh libevacx_head.so libevacx.so libevacx_b.so || exit 1
