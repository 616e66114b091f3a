set -o pipefail
mkdir -p gpurun_out
for cap in 256 384 512; do for mn in 300 450 569; do
  EVX_HEAVY_CAP=$cap EVX_HEAVY_MIN=$mn timeout -k 10 200 python bench.py --no-cpu --mode env --warmup 1300 --steps 100 > gpurun_out/tune_${cap}_${mn}.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tune_${cap}_${mn}.json'));print('cap $cap min $mn', round(d['env_step_kernel_ms'],4), round(d['ms_per_step'],4))"
done; done
