#!/bin/bash
# learn chain under env-var settings: tools/gpu_envsweep_learn.sh VAR "v1 v2 ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
VAR=$1
for n in $2; do
  echo "== $VAR=$n"
  env $VAR=$n KT_TOP=${KT_TOP:-9} bash $R/tools/gpu_ktrace.sh ${VAR}_$n python3 $R/tools/learn_bench.py 32768 20 || exit 1
done
