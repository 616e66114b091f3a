#!/bin/bash
# big-grid env kernels (bitmaps in global scratch): env parity suites, cfg4 bench line, cfg4 stamps, headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py tests/test_dropin_gpu.py > gpurun_out/bigg_tests.log 2>&1 || { tail -30 gpurun_out/bigg_tests.log; exit 1; }
tail -2 gpurun_out/bigg_tests.log
bash tools/gpu_configs.sh || exit 1
timeout -k 10 300 python tools/stamp_probe.py --grid 256 --people 9102 --robots 1 --envs 8192 --warmup 300 --stagger 300 > gpurun_out/stamps_cfg4.txt 2>&1 || { tail gpurun_out/stamps_cfg4.txt; exit 1; }
head -12 gpurun_out/stamps_cfg4.txt
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b_head.json 2> gpurun_out/b_head.err || { tail -5 gpurun_out/b_head.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_head.json'));print('headline %.3fM ms %.3f env %.3f' % (d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms']))"
