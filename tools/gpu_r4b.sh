#!/bin/bash
# act / learn / env parity suites on the current build, then the act microbench and a bench line
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_qmlp_x3_gpu.py tests/test_target_table_gpu.py tests/test_qmlp_gpu.py tests/test_act_rowperm_gpu.py \
    tests/test_draws_gpu.py tests/test_learner_golden_gpu.py tests/test_trainer_gpu.py tests/test_env_gpu.py \
    tests/test_bench_scale_gpu.py tests/test_dropin_gpu.py > gpurun_out/r4b/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4b/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/r4b/tests.log | head -30; exit $rc; }
timeout -k 10 200 python tools/act3_bench.py --table-frac 1.0 > gpurun_out/r4b/act.txt 2>&1 && grep "per act" gpurun_out/r4b/act.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --start-steps 0 > gpurun_out/r4b/bench.json 2> gpurun_out/r4b/bench.err || { tail gpurun_out/r4b/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4b/bench.json')); print('value', d['value']/1e6, 'ms', d['ms_per_step'], 'env', d['env_step_kernel_ms'], 'learn', d['learn_ms'], 'env_only', d['env_only_steps_per_s']/1e6)"
