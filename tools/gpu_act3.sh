#!/bin/bash
# x3 act microbenchmark + SQ counters of qact3_kernel (two PMC passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/act3
mkdir -p "$OUT"
timeout -k 10 120 python3 "$R/tools/act3_bench.py" $ACTARGS > "$OUT/bench.txt" 2>&1 || exit 1
cat "$OUT/bench.txt"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-include-regex qact3h --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU \
    -d "$OUT/p1" -o run --output-format csv -- python3 "$R/tools/act3_bench.py" --iters 3 $ACTARGS > "$OUT/p1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-include-regex qact3h --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    -d "$OUT/p2" -o run --output-format csv -- python3 "$R/tools/act3_bench.py" --iters 3 $ACTARGS > "$OUT/p2.log" 2>&1 || exit 1
for p in p1 p2; do
  f=$(find "$OUT/$p" -name "*counter_collection.csv" | head -1)
  python3 "$R/tools/sq_summary.py" "$f" qact3h_kernel
done
