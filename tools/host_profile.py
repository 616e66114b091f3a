#!/usr/bin/env python3
"""cProfile of VecTrainer.step()'s host side (Python + ctypes + HIP launch calls) at cfg2
(64x64, 569 people, 8 robots, 4096 envs, batch 4096, strict schedule): the functions whose
own time dominates, per step."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))
import torch  # noqa: E402

from evacx.env import DeviceLayout  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402
from evacx.trainer import VecTrainer  # noqa: E402

lay = DeviceLayout(build_tables(synthetic(64, 64, 8)), 569)
tr = VecTrainer(lay, 4096, batch=4096)
for _ in range(300):
    tr.step()
tr.sync()
torch.cuda.synchronize()
N = 300
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    tr.step()
pr.disable()
tr.sync()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime")
rows = sorted(st.stats.items(), key=lambda kv: -kv[1][2])[:30]
tot = sum(v[2] for v in st.stats.values())
print(f"host total {1e6 * tot / N:.0f} us per step (profiled)")
for (f, line, name), (cc, nc, tt, ct, _) in rows:
    print(f"{1e6 * tt / N:8.1f} us/step own  {nc / N:6.1f} calls/step  {os.path.basename(f)}:{line} {name}")
