#!/bin/bash
# A/B of act builds: tools/gpu_actab.sh lib1.so lib2.so ... (the in-tree libevacx.so first and last)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/actab"
for L in dqn-marl_amd/evacx/libevacx.so "$@" dqn-marl_amd/evacx/libevacx.so; do
  for f in ${FRACS:-0 0.85 1.0}; do
    EVX_LIB=$R/$L timeout -k 10 120 python3 "$R/tools/act3_bench.py" --table-frac $f > "$R/gpurun_out/actab/o.txt" 2>&1 || { cat "$R/gpurun_out/actab/o.txt"; exit 1; }
    echo "$(basename $L) frac $f: $(tail -1 "$R/gpurun_out/actab/o.txt")"
  done
done
