#!/bin/bash
# A/B of the x3 GEMM's k-pair staging (experiment lib): conv/learner numerics with it, conv microbenchmark both, cfg4 line with it
set -o pipefail
O=gpurun_out/pair; mkdir -p $O
X=$(pwd)/dqn-marl_amd/evacx/libevacx_pair.so
EVX_LIB=$X timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_qnet_gpu.py tests/test_learner_golden_gpu.py tests/test_qmix_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo control; timeout -k 10 120 python tools/conv_bench.py || exit 1
echo pair; EVX_LIB=$X timeout -k 10 120 python tools/conv_bench.py || exit 1
EVX_LIB=$X timeout -k 10 500 python bench.py --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 20 --other-steps 0 --start-steps 0 --batch 1024 > $O/b_cfg4.json 2>$O/b_cfg4.err || { tail -5 $O/b_cfg4.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_cfg4.json'));print('cfg4 pair value %.3fM env-steps/s, ms %.3f, env kernel %.3f ms, learn %.3f' % (d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms']))"
