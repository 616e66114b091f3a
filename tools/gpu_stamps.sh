#!/bin/bash
# Per-phase env-step stamps (normal and EVX_PROFILE builds), heavy-first order on.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps.txt 2>&1 || { tail gpurun_out/stamps.txt; exit 1; }
EVACX_LIB=libevacx_prof.so timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps_prof.txt 2>&1 || { tail gpurun_out/stamps_prof.txt; exit 1; }
cat gpurun_out/stamps.txt gpurun_out/stamps_prof.txt
