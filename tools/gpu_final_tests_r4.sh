#!/bin/bash
# round-4 GPU test suite (the driver's -m gpu run), log under gpurun_out/final_r4/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final_r4; mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && grep -E "^E |FAILED|Error" $OUT/tests.log | head -30
exit $rc
