#!/bin/bash
# fc1 timing experiments: EVX_FC1_DIAG 0 (normal), 1 (no table reads), 2 (no MFMA), 4 (no H1 stores), 7 (none)
set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2 4 3 7; do
  echo "diag $d"
  EVX_FC1_DIAG=$d timeout -k 10 120 python tools/qmlp_bench.py 2>&1 | grep -E "fc1 only|act"
done
