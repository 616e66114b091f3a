#!/bin/bash
# round 5: replay push, the next orders and the learn batch in one launch (one group, uniform replay)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5j; rm -rf $OUT; mkdir -p $OUT
cd $R
DEF="tests/test_order_gpu.py tests/test_trainer_gpu.py tests/test_concurrency_gpu.py tests/test_distributed_gpu.py tests/test_draws_gpu.py tests/test_bench_dist_gpu.py"
timeout -k 10 900 python -u -m pytest ${TESTS:-$DEF} -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/tests.log | head -40; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 > $OUT/b_$i.json 2> $OUT/b_$i.err || { tail -5 $OUT/b_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$i.json')); print('value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn', d['learn_ms'], 'alone', d['learn_alone_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { tail $OUT/trace_bench.err; exit 1; }
python3 $R/tools/step_gaps.py $OUT/t > $OUT/step_gaps.txt 2>&1 || true
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/t
cd $R

