#!/bin/bash
# full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r2d/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2d/smoke.log 2>&1
echo "smoke rc=$?"
