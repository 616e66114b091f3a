#!/bin/bash
# x3 act microbench (524288 rows, table fraction 1.0): kernel trace + one SQ pass (tools/kstats.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/actprof_${1:-a}; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/tools/act3_bench.py --table-frac 1.0 --iters 8"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- $CMD > $OUT/t.log 2>&1 || { tail $OUT/t.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $SQ -d $OUT/sq -o run --output-format csv -- $CMD > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/gr -o run --output-format csv -- $CMD > $OUT/gr.log 2>&1 || { tail $OUT/gr.log; exit 1; }
grep "per act" $OUT/t.log
python3 $R/tools/kstats.py $OUT 5 | head -12
