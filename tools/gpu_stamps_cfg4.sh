#!/bin/bash
# Per-phase env-step stamps at cfg4's geometry (256x256, P 9102, R 1, 8192 envs, stationary mix)
set -o pipefail
mkdir -p gpurun_out
A="--grid 256 --people 9102 --robots 1 --envs 8192 --warmup 300 --stagger 300"
timeout -k 10 300 python tools/stamp_probe.py $A > gpurun_out/stamps_cfg4.txt 2>&1 || { tail gpurun_out/stamps_cfg4.txt; exit 1; }
EVACX_LIB=libevacx_prof.so timeout -k 10 300 python tools/stamp_probe.py $A > gpurun_out/stamps_cfg4_prof.txt 2>&1 || { tail gpurun_out/stamps_cfg4_prof.txt; exit 1; }
cat gpurun_out/stamps_cfg4.txt gpurun_out/stamps_cfg4_prof.txt
