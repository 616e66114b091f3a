#!/bin/bash
# env_step_kernel phase stamps: stationary mix and start of episode, plain and EVX_PROFILE builds
set -o pipefail
mkdir -p gpurun_out/r2f
timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/r2f/stamps_stationary.txt 2>&1 && \
timeout -k 10 200 python tools/stamp_probe.py --reset-all > gpurun_out/r2f/stamps_start.txt 2>&1 && \
EVACX_LIB=libevacx_prof.so timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/r2f/prof_stationary.txt 2>&1 && \
EVACX_LIB=libevacx_prof.so timeout -k 10 200 python tools/stamp_probe.py --reset-all > gpurun_out/r2f/prof_start.txt 2>&1
echo rc=$?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_floor_gpu.py > gpurun_out/r2f/floor.log 2>&1
echo floor rc=$?
