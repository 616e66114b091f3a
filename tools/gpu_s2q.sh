#!/bin/bash
# round 6 (session 2): env_step per-phase cycle shares at cfg3 (stationary mix, 32768 envs): normal build
# (phase stamps) and the EVX_PROFILE build (sub-phase accumulators); shares only, not wall time
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/s2q; mkdir -p $O
timeout -k 10 300 python3 tools/stamp_probe.py --envs 32768 > $O/env_phases_cfg3.txt 2>&1 || { tail $O/env_phases_cfg3.txt; exit 1; }
EVX_LIB=$R/dqn-marl_amd/evacx/libevacx_prof.so timeout -k 10 300 python3 tools/stamp_probe.py --envs 32768 > $O/env_subphases_cfg3.txt 2>&1 || { tail $O/env_subphases_cfg3.txt; exit 1; }
cat $O/env_phases_cfg3.txt $O/env_subphases_cfg3.txt
