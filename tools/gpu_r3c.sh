#!/bin/bash
# split learn step: its parity tests, the trainer / draw suites, then the default bench
set -o pipefail
O=gpurun_out/r3c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_split_learn_gpu.py \
  tests/test_draws_gpu.py tests/test_trainer_gpu.py "tests/test_bench_scale_gpu.py::test_x3_learn_at_bench_batch" \
  tests/test_distributed_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5
[ $rc -ne 0 ] && { tail -40 $O/pytest.log; exit $rc; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$O/bench.json')); print(d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms'], d['learn_alone_ms'], d['learn_split_rows'], d['other_schedule'], d['roofline']['frac'], d.get('roofline_learn',{}).get('frac'))"
