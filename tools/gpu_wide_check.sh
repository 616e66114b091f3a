set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_env_gpu.py -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
EVACX_LIB=$GRAFT_REPO_ROOT/dqn-marl_amd/evacx/libevacx_prof.so timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps_prof.txt 2>&1 || exit 1
for cap in 0 128 256; do
  EVX_HEAVY_CAP=$cap timeout -k 10 200 python bench.py --no-cpu --mode env > gpurun_out/tune_${cap}.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tune_${cap}.json'));print('cap $cap', round(d['env_step_kernel_ms'],4), round(d['ms_per_step'],4))"
done
