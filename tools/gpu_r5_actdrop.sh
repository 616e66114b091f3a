#!/bin/bash
# round 5: x3 act with and without its dropout epilogue (the hash's share of the act), 524288 rows, table path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for p in 0.1 0 0.1 0; do timeout -k 10 200 python3 tools/act3_bench.py --table-frac 1.0 --drop-p $p 2>&1 | tail -1 | sed "s/^/p=$p /"; done
