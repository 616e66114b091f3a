#!/bin/bash
# split-K workgroup target sweep of the learn chain
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for n in ${NS:-256 512 768 1024}; do
  echo "== EVX_KSPLIT_WG=$n"
  EVX_KSPLIT_WG=$n KT_TOP=9 bash $R/tools/gpu_ktrace.sh ks$n python3 $R/tools/learn_bench.py 32768 20 || exit 1
done
