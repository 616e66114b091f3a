#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/st32k
timeout -k 10 300 python tools/stamp_probe.py --envs 32768 > gpurun_out/st32k/stamps.txt 2>&1
echo rc=$?
cat gpurun_out/st32k/stamps.txt | grep -v Warning
