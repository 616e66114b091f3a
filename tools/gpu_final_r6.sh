#!/bin/bash
# round-6 evidence: GPU suite, the driver's default bench line, its kernel trace / stats and one
# step's timeline; logs under gpurun_out/<tag>/
# usage: tools/gpu_final_r6.sh TAG
set -o pipefail
TAG=${1:-final_r6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/tests.log | head -40; exit $rc; }
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('cfg3', 'value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn %.3f alone %.3f' % (d['learn_ms'], d['learn_alone_ms']), 'frac %.3f' % d['roofline']['frac'], 'act', d.get('roofline_act', {}).get('act_ms'))"
cd /tmp && export TMPDIR=/tmp
# (the traced run stops after the timed and instrumented training passes, so the trace's last steps
# are training steps for step_gaps.py)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { tail -5 $OUT/trace_bench.err; exit 1; }
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 $R/tools/step_gaps.py $OUT/t > $OUT/step_gaps.txt 2>&1 || true
python3 $R/tools/step_kstats.py $OUT/t 20 > $OUT/kernel_stats_timed_steps.txt 2>&1 || true
rm -rf $OUT/t
