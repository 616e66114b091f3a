#!/bin/bash
# round-5 evidence: GPU suite, the driver's default bench line (no flags), its kernel trace / stats and step
# timeline, and the other BASELINE configs' lines with their cpu_baseline; everything under gpurun_out/$TAG
set -o pipefail
TAG=${1:-final_r5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
cd $R
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
  rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/tests.log | head -40; exit $rc; }
fi
summ() { python3 -c "
import json; d=json.load(open('$1')); c=d.get('cpu_baseline') or {}
print('$2', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn', d.get('learn_ms'), 'frac %.3f' % d['roofline']['frac'], 'cpu', c.get('value'), c.get('cores'))"; }
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
summ $OUT/bench.json cfg3
timeout -k 10 300 python3 bench.py --grid 64 --people 569 --robots 8 --envs 4096 --steps 300 --warmup 20 \
    > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err || { tail -5 $OUT/bench_cfg2.err; exit 1; }
summ $OUT/bench_cfg2.json cfg2
timeout -k 10 400 python3 bench.py --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 \
    > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -5 $OUT/bench_cfg5.err; exit 1; }
summ $OUT/bench_cfg5.json cfg5
timeout -k 10 600 python3 bench.py --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 \
    --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 20 --other-steps 0 --start-steps 0 --batch 1024 \
    --cpu-envs 128 --cpu-steps 100 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err || { tail -5 $OUT/bench_cfg4.err; exit 1; }
summ $OUT/bench_cfg4.json cfg4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { tail -5 $OUT/trace_bench.err; exit 1; }
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 $R/tools/step_gaps.py $OUT/t > $OUT/step_gaps.txt 2>&1 || true
rm -rf $OUT/t
