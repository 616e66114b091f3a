#!/bin/bash
# every GPU suite (one pytest process) + the default bench without the CPU leg
set -o pipefail
mkdir -p gpurun_out/all
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/all/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/all/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/all/bench.json 2> gpurun_out/all/bench.err
echo "bench rc=$?"; python -c "
import json; d=json.load(open('gpurun_out/all/bench.json')); print(d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms'], d['other_schedule'], d['env_only_steps_per_s']/1e6, d['start_phase'], d['roofline']['frac'])"
