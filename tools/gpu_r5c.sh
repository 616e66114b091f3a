#!/bin/bash
# round 5: transposed H1 planes in the x3 act (A/B against libevacx_oldact.so), fused orders, groups 2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5c; rm -rf $OUT; mkdir -p $OUT
cd $R
DEF="tests/test_qmlp_x3_gpu.py tests/test_target_table_gpu.py tests/test_bench_scale_gpu.py tests/test_learner_golden_gpu.py
  tests/test_qmlp_gpu.py tests/test_order_gpu.py tests/test_trainer_gpu.py tests/test_concurrency_gpu.py tests/test_distributed_gpu.py"
timeout -k 10 900 python -u -m pytest ${TESTS:-$DEF} -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/tests.log | head -40; exit $rc; }
for i in 1 2; do
  for v in new old; do
    L=""; [ $v = old ] && L="$R/dqn-marl_amd/evacx/libevacx_oldact.so"
    EVX_LIB=$L timeout -k 10 120 python3 tools/act3_bench.py --table-frac 1.0 > $OUT/act_${v}_$i.txt 2>&1 || { tail $OUT/act_${v}_$i.txt; exit 1; }
    echo "$v $(tail -1 $OUT/act_${v}_$i.txt)"
  done
done
for v in new old; do
  L=""; [ $v = old ] && L="$R/dqn-marl_amd/evacx/libevacx_oldact.so"
  EVX_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --env-steps 0 --start-steps 0 > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -5 $OUT/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn', d['learn_ms'], 'alone', d['learn_alone_ms'])"
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --groups 2 --env-steps 0 --start-steps 0 --other-steps 0 > $OUT/b_g2.json 2> $OUT/b_g2.err || { tail -5 $OUT/b_g2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_g2.json')); print('groups2 value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn', d['learn_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 \
    --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { tail $OUT/trace_bench.err; exit 1; }
python3 $R/tools/step_timeline.py $OUT/t 60 > $OUT/timeline.txt 2>&1 || true
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/t
