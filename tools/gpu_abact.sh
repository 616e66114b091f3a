#!/bin/bash
# In-box A/B of act builds (EVX_LIB): the act microbench at 524288 rows, interleaved, for each library
# named on the command line (files under dqn-marl_amd/evacx/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=$R/dqn-marl_amd/evacx
for i in 1 2 3; do
  for lib in "$@"; do
    echo -n "$lib: "; EVX_LIB=$L/$lib timeout -k 10 120 python tools/act3_bench.py --table-frac 1.0 2>&1 | tail -1 || exit 1
  done
done
