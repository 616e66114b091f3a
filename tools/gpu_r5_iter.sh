#!/bin/bash
# round-5 iteration: selected GPU tests, the default bench line, the step's kernel timeline
# usage: tools/gpu_r5_iter.sh TAG "pytest selection" [bench args...]
set -o pipefail
TAG=$1; SEL=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
cd $R
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest $SEL -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/tests.log | head -40; exit $rc; }
fi
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn', d['learn_ms'], 'alone', d['learn_alone_ms'], 'frac %.3f' % d['roofline']['frac'], 'other', d['other_schedule'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 "$@" > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { tail $OUT/trace_bench.err; exit 1; }
python3 $R/tools/step_timeline.py $OUT/t 60 > $OUT/timeline.txt 2>&1 || true
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/t
