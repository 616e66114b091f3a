set -o pipefail
mkdir -p gpurun_out
for mp in -1 0; do for lp in -1 0; do
EVX_MAIN_PRIO=$mp EVX_LEARN_PRIO=$lp timeout -k 10 300 python bench.py --no-cpu --env-steps 0 --strict-steps 0 > gpurun_out/p.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/p.json'));print('main $mp learn $lp', round(d['ms_per_step'],4), round(d['env_step_kernel_ms'],4), round(d['learn_ms'],4))"
done; done
