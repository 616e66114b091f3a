#!/bin/bash
# per-phase stamps of env_step_kernel at 32768 envs (stationary mix): normal and EVX_PROFILE builds
set -o pipefail
mkdir -p gpurun_out/st4
timeout -k 10 300 python tools/stamp_probe.py --envs 32768 > gpurun_out/st4/stamps.txt 2>&1
rc=$?
grep -v Warning gpurun_out/st4/stamps.txt
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROF" ]; then
  EVX_LIB=$PWD/dqn-marl_amd/evacx/libevacx_prof.so timeout -k 10 300 python tools/stamp_probe.py --envs 32768 > gpurun_out/st4/stamps_prof.txt 2>&1
  rc=$?
  grep -v Warning gpurun_out/st4/stamps_prof.txt
fi
exit $rc
