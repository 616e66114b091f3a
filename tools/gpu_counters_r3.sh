#!/bin/bash
# Round-3 counter evidence for the three kernels of the step, each in its own PMC passes
# (kernel trace + one SQ pass + one GRBM pass; summarised by tools/kstats.py):
#   learn chain  -- tools/learn_bench.py at B = 32768 (qfc1, qfc23, qact3h target, bwd_mid, gemm_tn, ...)
#   x3 act       -- tools/act3_bench.py at 524288 rows, table fraction 1.0 (qact3h_kernel)
#   env.step     -- bench.py --mode env (env_step_kernel at 32768 envs, stationary mix)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
run3() {  # name, command...
  local OUT=$R/gpurun_out/cnt_$1; shift; rm -rf $OUT; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- "$@" > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; return 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ -d $OUT/sq -o run --output-format csv -- "$@" > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; return 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/gr -o run --output-format csv -- "$@" > $OUT/gr.log 2>&1 || { tail $OUT/gr.log; return 1; }
  python3 $R/tools/kstats.py $OUT > $OUT/kstats.txt 2>&1; head -25 $OUT/kstats.txt
  # keep the summaries only (the raw per-dispatch CSVs of 1300 env launches exceed gpurun's 64 MiB)
  find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
  rm -rf $OUT/t $OUT/sq $OUT/gr
}
run3 learn python3 $R/tools/learn_bench.py 32768 10 && \
run3 act python3 $R/tools/act3_bench.py --table-frac 1.0 && \
run3 env python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0
