#!/bin/bash
# x3 act/forward change: x3 + qmlp + bench-scale + trainer suites, then the act microbench and the learn chain
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/act6; mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_qmlp_x3_gpu.py tests/test_qmlp_gpu.py \
  tests/test_bench_scale_gpu.py tests/test_trainer_gpu.py tests/test_qnet_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for f in 0 1.0; do
  timeout -k 10 120 python3 tools/act3_bench.py --table-frac $f > "$OUT/h_$f.txt" 2>&1 || { cat "$OUT/h_$f.txt"; exit 1; }
  echo "frac $f: $(tail -1 "$OUT/h_$f.txt")"
done
timeout -k 10 120 python3 tools/learn_bench.py 32768 20 2>&1 | grep learn
