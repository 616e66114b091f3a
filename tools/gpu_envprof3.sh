#!/bin/bash
# env_step_kernel at the bench's stationary 32768-env mix: phase stamps (normal and EVX_PROFILE
# builds), SQ instruction mix and wait breakdown of the timed launches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/envprof_${1:-a}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/stamp_probe.py --envs 32768 > $OUT/stamps.txt 2>&1 || { tail $OUT/stamps.txt; exit 1; }
EVACX_LIB=libevacx_prof.so timeout -k 10 300 python3 $R/tools/stamp_probe.py --envs 32768 > $OUT/stamps_prof.txt 2>&1 || { tail $OUT/stamps_prof.txt; exit 1; }
X="--mode env --steps 10 --warmup 2 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0"
timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex env_step_kernel --kernel-iteration-range "[1300-1320]" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/mix -o run --output-format csv -- python3 $R/bench.py $X > $OUT/mix.log 2>&1 || { tail $OUT/mix.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex env_step_kernel --kernel-iteration-range "[1300-1320]" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $OUT/sq -o run --output-format csv -- python3 $R/bench.py $X > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
grep -v Warn $OUT/stamps.txt | head -30
grep -v Warn $OUT/stamps_prof.txt | tail -26
for d in mix sq; do python3 $R/tools/sq_summary.py $(find $OUT/$d -name "*counter_collection.csv" | head -1); done
