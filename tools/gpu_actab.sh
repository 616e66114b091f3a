#!/bin/bash
# act microbench A/B over experiment builds (EVX_LIB): default, then each libevacx_<tag>.so given
set -o pipefail
for tag in default "$@"; do
  if [ "$tag" = default ]; then L=""; else L="EVX_LIB=$PWD/dqn-marl_amd/evacx/libevacx_$tag.so"; fi
  echo -n "$tag: "; env $L timeout -k 10 200 python tools/act3_bench.py --table-frac 1.0 2>&1 | grep "per act" || exit 1
done
