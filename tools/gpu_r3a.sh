#!/bin/bash
# round 3: the new bench-scale parity tests, the deterministic split-K and without-replacement
# sampler, bench.py's world-2 gloo branch; then the whole GPU suite and smoke
set -o pipefail
O=gpurun_out/r3a; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_bench_scale_gpu.py tests/test_draws_gpu.py tests/test_gemm_epilogue_gpu.py \
    tests/test_qnet_gpu.py tests/test_bench_dist_gpu.py > $O/new.log 2>&1 || { tail -40 $O/new.log; exit 1; }
tail -3 $O/new.log
timeout -k 10 900 $T tests -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo ALLOK
