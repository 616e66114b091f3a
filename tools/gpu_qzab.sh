#!/bin/bash
# qdz1 ablations: per-kernel time of the split backward under each experiment library
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for L in "$@"; do
  echo "== $L"
  EVX_SPLIT_MID=1 EVX_LIB=$R/$L KT_TOP=6 bash $R/tools/gpu_ktrace.sh $(basename $L .so) python3 $R/tools/learn_bench.py 32768 10 || exit 1
done
