set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision bf16 > gpurun_out/r2a/bf16_strict.json 2> gpurun_out/r2a/bf16_strict.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision bf16 --phase start --no-cpu --other-steps 0 --env-steps 0 > gpurun_out/r2a/bf16_start.json 2> gpurun_out/r2a/bf16_start.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r2a/f32_slow.json 2> gpurun_out/r2a/f32_slow.err
echo rc=$?
