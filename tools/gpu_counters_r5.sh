#!/bin/bash
# Round-5 counter evidence (every pass its own rocprofv3 run, counter limits per pass respected):
#   env   -- env_step_kernel, bench.py --mode env at cfg3 (32768 envs, stationary mix): trace, two SQ
#            passes, GRBM, FETCH_SIZE, WRITE_SIZE -> gpurun_out/cnt5_env/env_counters.json
#   learn -- tools/learn_bench.py at B = 32768 (tables) and 4096: trace + SQ + GRBM per kernel (kstats)
#   act   -- tools/act3_bench.py, 524288 rows, table fraction 1.0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
SQ2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
prof() {  # dir, pmc (or "" for trace), command...
  local D=$1 P=$2; shift 2
  if [ -z "$P" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- "$@" > $D.log 2>&1 || { tail $D.log; return 1; }
  else
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P -d $D -o run --output-format csv -- "$@" > $D.log 2>&1 || { tail $D.log; return 1; }
  fi
}
OUT=$R/gpurun_out/cnt5_env; rm -rf $OUT; mkdir -p $OUT
CMD="python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0"
prof $OUT/t "" $CMD && prof $OUT/sq "$SQ" $CMD && prof $OUT/sq2 "$SQ2" $CMD && prof $OUT/gr "GRBM_GUI_ACTIVE GRBM_COUNT" $CMD && \
  prof $OUT/fe FETCH_SIZE $CMD && prof $OUT/wr WRITE_SIZE $CMD || exit 1
python3 $R/tools/kstats.py $OUT > $OUT/kstats.txt 2>&1; head -4 $OUT/kstats.txt
python3 $R/tools/env_counters.py $OUT > $OUT/env_counters.json 2>&1; cat $OUT/env_counters.json
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/t $OUT/sq $OUT/sq2 $OUT/gr $OUT/fe $OUT/wr
for w in "learn:python3 $R/tools/learn_bench.py 32768 10 table" "learn4k:python3 $R/tools/learn_bench.py 4096 20" \
         "act:python3 $R/tools/act3_bench.py --table-frac 1.0"; do
  n=${w%%:*}; c=${w#*:}
  OUT=$R/gpurun_out/cnt5_$n; rm -rf $OUT; mkdir -p $OUT
  prof $OUT/t "" $c && prof $OUT/sq "$SQ" $c && prof $OUT/gr "GRBM_GUI_ACTIVE GRBM_COUNT" $c || exit 1
  python3 $R/tools/kstats.py $OUT > $OUT/kstats.txt 2>&1; echo "== $n"; head -14 $OUT/kstats.txt
  find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
  rm -rf $OUT/t $OUT/sq $OUT/gr
done
