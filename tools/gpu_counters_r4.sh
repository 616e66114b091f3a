#!/bin/bash
# Round-4 SQ / GRBM counters (kernel trace + one SQ pass + one GRBM pass each; tools/kstats.py) of
#   learn chain -- tools/learn_bench.py at B = 32768 with both nets' act tables (the trainer's path)
#   x3 act     -- tools/act3_bench.py at 524288 rows, table fraction 1.0 (qact3h_kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
run3() {  # name, command...
  local OUT=$R/gpurun_out/cnt4_$1; shift; rm -rf $OUT; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- "$@" > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; return 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ -d $OUT/sq -o run --output-format csv -- "$@" > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; return 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/gr -o run --output-format csv -- "$@" > $OUT/gr.log 2>&1 || { tail $OUT/gr.log; return 1; }
  python3 $R/tools/kstats.py $OUT > $OUT/kstats.txt 2>&1; head -14 $OUT/kstats.txt
  find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
  rm -rf $OUT/t $OUT/sq $OUT/gr
}
run3 learn python3 $R/tools/learn_bench.py 32768 10 table && \
run3 act python3 $R/tools/act3_bench.py --table-frac 1.0
