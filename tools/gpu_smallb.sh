#!/bin/bash
# learn chain at the cfg2 / cfg5 / cfg3 batches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for B in ${BS:-4096 8192 32768}; do
  echo "== B=$B"
  KT_TOP=${KT_TOP:-9} bash $R/tools/gpu_ktrace.sh sb python3 $R/tools/learn_bench.py $B 30 || exit 1
done
