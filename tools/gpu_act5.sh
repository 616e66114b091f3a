#!/bin/bash
# x3 act: parity tests (64-row tiles), then microbench of 64- vs 128-row tiles at three table fractions
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/act5; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_qmlp_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for f in 0 0.85 1.0; do
  timeout -k 10 120 python3 tools/act3_bench.py --table-frac $f > "$OUT/h_$f.txt" 2>&1 || { cat "$OUT/h_$f.txt"; exit 1; }
  EVX_ACT3_FULLTILE=1 timeout -k 10 120 python3 tools/act3_bench.py --table-frac $f > "$OUT/f_$f.txt" 2>&1 || { cat "$OUT/f_$f.txt"; exit 1; }
  echo "frac $f: 64-row $(tail -1 "$OUT/h_$f.txt" | cut -d: -f2 | cut -d, -f1) | 128-row $(tail -1 "$OUT/f_$f.txt" | cut -d: -f2 | cut -d, -f1)"
done
