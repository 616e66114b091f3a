set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps.txt 2>&1 || exit 1
EVACX_LIB=$GRAFT_REPO_ROOT/dqn-marl_amd/evacx/libevacx_prof.so timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps_prof.txt 2>&1 || exit 1
for cap in 0 128 256 512; do for mn in 300 569 1000; do
  EVX_HEAVY_CAP=$cap EVX_HEAVY_MIN=$mn timeout -k 10 200 python bench.py --no-cpu --mode env --warmup 1300 --steps 100 > gpurun_out/tune_${cap}_${mn}.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tune_${cap}_${mn}.json'));print('cap $cap min $mn', round(d['env_step_kernel_ms'],4), round(d['ms_per_step'],4))"
done; done
