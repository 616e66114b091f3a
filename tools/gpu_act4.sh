#!/bin/bash
# x3 act: parity tests, microbench at three table fractions, stamp timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/act4
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_qmix_golden_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -3 "$OUT/tests.txt"
for f in 0 0.85 1.0; do
  timeout -k 10 120 python3 tools/act3_bench.py --table-frac $f > "$OUT/bench_$f.txt" 2>&1 || { cat "$OUT/bench_$f.txt"; exit 1; }
  echo "frac $f: $(tail -2 "$OUT/bench_$f.txt")"
done
timeout -k 10 120 python3 tools/act_stamps.py 1.0 > "$OUT/stamps.txt" 2>&1 || { cat "$OUT/stamps.txt"; exit 1; }
cat "$OUT/stamps.txt"
