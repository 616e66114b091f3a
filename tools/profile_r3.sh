#!/bin/bash
# Round-3 evidence on a GPU box: tools/profile_r2.sh (driver's bench command, kernel traces of the
# stationary and start phases, env_step FETCH/WRITE PMC passes) plus the other BASELINE configs
# as bench lines (cfg2, cfg4 = conv Q-net, cfg5 = prioritized replay), all under gpurun_out/prof_<tag>.
set -o pipefail
TAG=${1:-r3a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/profile_r2.sh" "$TAG" || exit $?
OUT=$R/gpurun_out/prof_$TAG
cd "$R"
timeout -k 10 300 python3 bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 --env-steps 0 \
    > "$OUT/bench_cfg2.json" 2> "$OUT/bench_cfg2.err" || { tail -5 "$OUT/bench_cfg2.err"; exit 1; }
echo "cfg2 done"
timeout -k 10 400 python3 bench.py --no-cpu --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 --env-steps 0 \
    > "$OUT/bench_cfg5.json" 2> "$OUT/bench_cfg5.err" || { tail -5 "$OUT/bench_cfg5.err"; exit 1; }
echo "cfg5 done"
timeout -k 10 500 python3 bench.py --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 \
    --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 20 --other-steps 0 --start-steps 0 --batch 1024 \
    > "$OUT/bench_cfg4.json" 2> "$OUT/bench_cfg4.err" || { tail -5 "$OUT/bench_cfg4.err"; exit 1; }
echo "cfg4 done"
