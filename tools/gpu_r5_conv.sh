#!/bin/bash
# round 5: conv2 / conv3 forward with the weights in registers (conv3x3_wreg_kernel): conv parity
# tests, then the cfg4 bench line and its step timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5conv; rm -rf $OUT; mkdir -p $OUT
cd $R
T="tests/test_qnet_gpu.py tests/test_bench_scale_gpu.py tests/test_concurrency_gpu.py tests/test_learner_golden_gpu.py tests/test_gemm_epilogue_gpu.py tests/test_dropin_gpu.py"
timeout -k 10 900 python -u -m pytest ${TESTS:-$T} -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/tests.log | head -40; exit $rc; }
C4="--grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 5 --age-steps 300 --stagger 300 --batch 1024"
timeout -k 10 500 python3 bench.py --no-cpu $C4 --steps 10 --env-steps 0 --other-steps 0 --start-steps 0 > $OUT/b_cfg4.json 2> $OUT/b_cfg4.err || { tail -5 $OUT/b_cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_cfg4.json')); print('cfg4 value %.3f M' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], 'env %.3f' % d['env_step_kernel_ms'], 'learn', d['learn_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 $R/bench.py --no-cpu $C4 --steps 4 \
    --env-steps 0 --other-steps 0 --start-steps 0 > $OUT/trace_cfg4.json 2> $OUT/trace_cfg4.err || { tail $OUT/trace_cfg4.err; exit 1; }
python3 $R/tools/step_timeline.py $OUT/t 70 > $OUT/timeline_cfg4.txt 2>&1 || true
find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_cfg4.csv \;
rm -rf $OUT/t
