#!/bin/bash
# round-2 final evidence: full GPU suite + smoke, profile_r2.sh (driver command, traces, PMC) under TAG,
# per-config bench lines (cfg2, cfg5, cfg4 conv) and the cfg4 kernel trace
set -o pipefail
TAG=${1:-r2e}
O=gpurun_out/final_$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo smoke ok
bash tools/profile_r2.sh $TAG || exit $?
timeout -k 10 300 python bench.py --no-cpu --grid 64 --people 569 --robots 8 --envs 4096 > $O/b_cfg2.json 2>$O/b_cfg2.err || { tail -5 $O/b_cfg2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --replay prioritized --robots 32 --envs 8192 --replay-capacity 4194304 > $O/b_cfg5.json 2>$O/b_cfg5.err || { tail -5 $O/b_cfg5.err; exit 1; }
timeout -k 10 500 python bench.py --no-cpu --grid 256 --people 9102 --robots 1 --envs 8192 --qnet conv --precision f32 --warmup 5 --age-steps 300 --stagger 300 --steps 10 --env-steps 20 --other-steps 0 --start-steps 0 --batch 1024 > $O/b_cfg4.json 2>$O/b_cfg4.err || { tail -5 $O/b_cfg4.err; exit 1; }
bash tools/gpu_cfg4prof.sh || exit $?
echo ALLOK
