#!/bin/bash
# Round-6 counter records of env_step_kernel for bench.py's roofline objects (roofline_hbm.traffic,
# roofline_issue): per config, bench.py --mode env on that config's workload under three rocprofv3 runs
# (kernel trace; SQ x8 + GRBM x2 + FETCH_SIZE; WRITE_SIZE -- per-block counter limits respected) ->
# gpurun_out/r6cnt/env_counters_stationary_<cfg>.json (tools/env_counters.py: SQ ratios, instructions per
# wave, clock, HBM bytes per env-step). Usage: gpu_r6_counters.sh cfg3 [cfg2 cfg5 cfg4]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r6cnt; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
for cfg in "$@"; do
  case $cfg in
    cfg3) A="--envs 32768"; E=32768; G=128; P=2276; RB=16 ;;
    cfg2) A="--grid 64 --people 569 --robots 8 --envs 4096"; E=4096; G=64; P=569; RB=8 ;;
    cfg5) A="--robots 32 --envs 8192 --replay prioritized --replay-capacity 4194304"; E=8192; G=128; P=2276; RB=32 ;;
    cfg4) A="--grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --age-steps 300 --stagger 300 --batch 1024"; E=8192; G=256; P=9102; RB=1 ;;
    *) echo "unknown $cfg"; exit 2 ;;
  esac
  CMD="python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu --env-steps 0 --other-steps 0 --start-steps 0 $A"
  D=$OUT/$cfg; rm -rf $D; mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o run --output-format csv -- $CMD > $D/t.log 2>&1 || { tail $D/t.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ GRBM_GUI_ACTIVE GRBM_COUNT FETCH_SIZE -d $D/sq -o run --output-format csv -- $CMD > $D/sq.log 2>&1 || { tail $D/sq.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $D/wr -o run --output-format csv -- $CMD > $D/wr.log 2>&1 || { tail $D/wr.log; exit 1; }
  python3 $R/tools/env_counters.py $D $E stationary $G $P $RB > $OUT/env_counters_stationary_$cfg.json 2>&1
  cat $OUT/env_counters_stationary_$cfg.json
  find $D/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_env_$cfg.csv \;
  rm -rf $D
done
