#!/bin/bash
# Round-6 counter evidence for the MFMA kernels (every pass its own rocprofv3 run, counter limits per
# pass respected): kernel trace + one SQ pass + one GRBM pass per workload, summarised per kernel by
# tools/kstats.py (wait / issue fractions, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock x
# duration), clock = GRBM_GUI_ACTIVE / 8 XCDs / duration):
#   act     -- tools/act3_bench.py, 524288 rows, table fraction 1.0 (the persistent x3 act)
#   learn   -- tools/learn_bench.py 32768 10 table (cfg3's learn)
#   learn8k -- tools/learn_bench.py 8192 10 table (cfg5's learn: the paired table-path forward)
#   learn4k -- tools/learn_bench.py 4096 20 (cfg2's learn)
# -> gpurun_out/cnt6_<name>/kstats.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
prof() {  # dir, pmc (or "" for trace), command...
  local D=$1 P=$2; shift 2
  if [ -z "$P" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- "$@" > $D.log 2>&1 || { tail $D.log; return 1; }
  else
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P -d $D -o run --output-format csv -- "$@" > $D.log 2>&1 || { tail $D.log; return 1; }
  fi
}
for w in "act:python3 $R/tools/act3_bench.py --table-frac 1.0" "learn:python3 $R/tools/learn_bench.py 32768 10 table" \
         "learn8k:python3 $R/tools/learn_bench.py 8192 10 table" "learn4k:python3 $R/tools/learn_bench.py 4096 20"; do
  n=${w%%:*}; c=${w#*:}
  OUT=$R/gpurun_out/cnt6_$n; rm -rf $OUT; mkdir -p $OUT
  prof $OUT/t "" $c && prof $OUT/sq "$SQ" $c && prof $OUT/gr "GRBM_GUI_ACTIVE GRBM_COUNT" $c || exit 1
  python3 $R/tools/kstats.py $OUT > $OUT/kstats.txt 2>&1; echo "== $n"; head -14 $OUT/kstats.txt
  find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
  rm -rf $OUT/t $OUT/sq $OUT/gr
done
