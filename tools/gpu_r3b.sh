#!/bin/bash
# trainer tests + smoke, the driver's bench command, a kernel trace of the headline
set -o pipefail
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_trainer_gpu.py > $O/trainer.log 2>&1 || { tail -30 $O/trainer.log; exit 1; }
tail -1 $O/trainer.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['env_step_kernel_ms'], d['learn_ms'], d['roofline']['frac'])"
bash tools/gpu_trace_head.sh > $O/trace.txt 2>&1 || { tail $O/trace.txt; exit 1; }
head -25 $O/trace.txt
