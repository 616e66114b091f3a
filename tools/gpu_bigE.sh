#!/bin/bash
# cfg3 as BASELINE.json states it on one GPU: 32768 envs (batch scaled with the envs) vs the 4096-env share
set -o pipefail
mkdir -p gpurun_out/bigE
timeout -k 10 400 python bench.py --envs 32768 --batch 32768 --replay-capacity 8388608 --steps 10 --warmup 3 --no-cpu --start-steps 0 --env-steps 20 > gpurun_out/bigE/e32k_b32k.json 2> gpurun_out/bigE/e32k_b32k.err
echo "e32k b32k rc=$?"
timeout -k 10 400 python bench.py --envs 16384 --batch 16384 --replay-capacity 4194304 --steps 10 --warmup 3 --no-cpu --start-steps 0 --env-steps 20 > gpurun_out/bigE/e16k_b16k.json 2> gpurun_out/bigE/e16k_b16k.err
echo "e16k rc=$?"
