#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
EVACX_LIB=libevacx_prof.so timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps_prof.txt 2>&1 || { tail gpurun_out/stamps_prof.txt; exit 1; }
grep -A40 "sub-phase" gpurun_out/stamps_prof.txt
