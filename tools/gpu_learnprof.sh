#!/bin/bash
# learn chain: timing, kernel trace, SQ counters (one pass) of tools/learn_bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/learnprof_${1:-a}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B=${2:-32768}
timeout -k 10 200 python3 $R/tools/learn_bench.py $B 20 > $OUT/bench.txt 2>&1 || { tail $OUT/bench.txt; exit 1; }
cat $OUT/bench.txt | grep learn
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/tools/learn_bench.py $B 20 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $OUT/sq -o run --output-format csv -- python3 $R/tools/learn_bench.py $B 5 > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/gr -o run --output-format csv -- python3 $R/tools/learn_bench.py $B 5 > $OUT/gr.log 2>&1 || { tail $OUT/gr.log; exit 1; }
python3 $R/tools/kstats.py $OUT
