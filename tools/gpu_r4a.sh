#!/bin/bash
# full GPU suite, then the step's kernel trace (tools/gpu_steptrace.sh) and the act's memory counters
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/gputest.log | tail -20; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_steptrace.sh r4a 30 && bash tools/gpu_actmem.sh env
