#!/bin/bash
# round 5: cfg4 env_step_kernel counters (SQ + FETCH/WRITE passes, bench --mode env) -> traffic record;
# cfg2 / cfg5 training-step kernel timelines (rocprofv3 kernel trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5cfg; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C4="--grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --age-steps 300 --stagger 300 --batch 1024"
CMD="python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0 $C4"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
SQ2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- $CMD > $OUT/t.log 2>&1 || { tail $OUT/t.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ -d $OUT/sq -o run --output-format csv -- $CMD > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ2 -d $OUT/sq2 -o run --output-format csv -- $CMD > $OUT/sq2.log 2>&1 || { tail $OUT/sq2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fe -o run --output-format csv -- $CMD > $OUT/fe.log 2>&1 || { tail $OUT/fe.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/wr -o run --output-format csv -- $CMD > $OUT/wr.log 2>&1 || { tail $OUT/wr.log; exit 1; }
python3 $R/tools/env_counters.py $OUT 8192 > $OUT/env_counters_cfg4.json 2>&1; cat $OUT/env_counters_cfg4.json
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_cfg4_env.csv \;
rm -rf $OUT/t $OUT/sq $OUT/sq2 $OUT/fe $OUT/wr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t2 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 --grid 64 --people 569 --robots 8 --envs 4096 > $OUT/trace_cfg2.json 2> $OUT/trace_cfg2.err || { tail $OUT/trace_cfg2.err; exit 1; }
python3 $R/tools/step_timeline.py $OUT/t2 40 > $OUT/timeline_cfg2.txt 2>&1 || true
find $OUT/t2 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_cfg2.csv \;
rm -rf $OUT/t2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t5 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 > $OUT/trace_cfg5.json 2> $OUT/trace_cfg5.err || { tail $OUT/trace_cfg5.err; exit 1; }
python3 $R/tools/step_timeline.py $OUT/t5 40 > $OUT/timeline_cfg5.txt 2>&1 || true
find $OUT/t5 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_cfg5.csv \;
rm -rf $OUT/t5
