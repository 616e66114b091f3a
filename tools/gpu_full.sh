#!/bin/bash
# full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/full/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/full/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1
echo "smoke rc=$?"
