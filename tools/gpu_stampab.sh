#!/bin/bash
# per-phase stamps A/B (default build vs libevacx_<tag>.so) ; args after the tag go to stamp_probe.py
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/stab
timeout -k 10 300 python tools/stamp_probe.py "$@" > gpurun_out/stab/default.txt 2>&1 || { tail gpurun_out/stab/default.txt; exit 1; }
EVX_LIB=$PWD/dqn-marl_amd/evacx/libevacx_$TAG.so timeout -k 10 300 python tools/stamp_probe.py "$@" > gpurun_out/stab/$TAG.txt 2>&1 || exit 1
echo "== default"; grep -v Warning gpurun_out/stab/default.txt | head -12; echo "== $TAG"; grep -v Warning gpurun_out/stab/$TAG.txt | head -12
