#!/bin/bash
# full GPU suite + the driver's bench command (no CPU leg)
set -o pipefail
O=gpurun_out/r2l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu > $O/b_head$i.json 2> $O/b_head$i.err || { tail -5 $O/b_head$i.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_head$i.json'));print('headline %.3fM ms %.3f env %.3f learn %.3f learn_frac %.4f' % (d['value']/1e6, d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms'], d['roofline_learn']['frac']))"
done
