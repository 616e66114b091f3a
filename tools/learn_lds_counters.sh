#!/bin/bash
# LDS counters of the learner kernels on a short training bench (one PMC pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/learnlds
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    -d "$OUT/p" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 40 --stagger 0 --no-cpu --env-steps 0 --strict-steps 0 > "$OUT/p.log" 2>&1 || { tail -5 "$OUT/p.log"; exit 1; }
f=$(find "$OUT/p" -name "*counter_collection.csv" | head -1)
for k in gemm_tn_kernel gemm_reduce qdz1_kernel qbwd3_kernel qfc23_kernel "qfc1_kernel<2" qact_kernel; do
  echo "== $k"; python3 "$R/tools/sq_summary.py" "$f" "$k" | grep -E "BANK|INSTS_LDS|WAIT_INST_LDS|WAVE_CYCLES  |SQ_WAVES"
done
