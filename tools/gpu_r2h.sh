#!/bin/bash
# full GPU suite + smoke + the driver's bench command (HEAD check after a container rebuild)
set -o pipefail
mkdir -p gpurun_out/r2h
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests -m gpu > gpurun_out/r2h/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r2h/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2h/smoke.log 2>&1 || exit $?
echo "smoke ok"
timeout -k 10 420 python bench.py --steps 20 --warmup 5 > gpurun_out/r2h/bench.json 2> gpurun_out/r2h/bench.err || exit $?
cat gpurun_out/r2h/bench.json | cut -c1-400
