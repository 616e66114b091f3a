#!/bin/bash
# round 6 (session 2): cfg2 kernel trace (per-kernel means over the last training steps, one step's timeline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2p; mkdir -p $O
A="--grid 64 --people 569 --robots 8 --envs 4096"
bash tools/gpu_prof.sh s2p/cfg2 -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 $A > $O/cfg2.txt 2>&1 || { tail $O/cfg2.txt; exit 1; }
python3 tools/step_kstats.py $O/cfg2 20 | head -30
python3 tools/step_gaps.py $O/cfg2 > $O/step_gaps.txt 2>&1; head -24 $O/step_gaps.txt
