#!/bin/bash
# Round-4 counter evidence for env_step_kernel (bench.py --mode env: 32768 envs, cfg3 stationary
# mix), every pass its own rocprofv3 run: kernel trace + stats, two SQ passes, GRBM, FETCH_SIZE,
# WRITE_SIZE. Summaries (tools/kstats.py, tools/env_counters.py) land in gpurun_out/cnt4_env/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/cnt4_env; rm -rf $OUT; mkdir -p $OUT
CMD="python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0 ${EXTRA:-}"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
SQ2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- $CMD > $OUT/t.log 2>&1 || { tail $OUT/t.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ -d $OUT/sq -o run --output-format csv -- $CMD > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ2 -d $OUT/sq2 -o run --output-format csv -- $CMD > $OUT/sq2.log 2>&1 || { tail $OUT/sq2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/gr -o run --output-format csv -- $CMD > $OUT/gr.log 2>&1 || { tail $OUT/gr.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fe -o run --output-format csv -- $CMD > $OUT/fe.log 2>&1 || { tail $OUT/fe.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/wr -o run --output-format csv -- $CMD > $OUT/wr.log 2>&1 || { tail $OUT/wr.log; exit 1; }
python3 $R/tools/kstats.py $OUT > $OUT/kstats.txt 2>&1; head -8 $OUT/kstats.txt
python3 $R/tools/env_counters.py $OUT > $OUT/env_counters.txt 2>&1; cat $OUT/env_counters.txt
# keep the summaries only (the raw per-dispatch CSVs of 1300 env launches exceed gpurun's 64 MiB)
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/t $OUT/sq $OUT/sq2 $OUT/gr $OUT/fe $OUT/wr
