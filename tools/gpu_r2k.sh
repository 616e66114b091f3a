#!/bin/bash
# big-grid LDS (validity bitmap from L2 in the fused reset, contest losers in global scratch): env parity suites, cfg4 line, headline
set -o pipefail
O=gpurun_out/r2k; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_env_gpu.py tests/test_dropin_gpu.py tests/test_layoutset_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python bench.py --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 20 --other-steps 0 --start-steps 0 --batch 1024 > $O/b_cfg4.json 2>$O/b_cfg4.err || { tail -5 $O/b_cfg4.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_cfg4.json'));print('cfg4 value %.3fM env-steps/s, ms %.3f, env kernel %.3f ms, frac %.3f' % (d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['roofline']['frac']))"
timeout -k 10 300 python bench.py --no-cpu > $O/b_head.json 2> $O/b_head.err || { tail -5 $O/b_head.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_head.json'));print('headline %.3fM ms %.3f env %.3f' % (d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms']))"
