#!/usr/bin/env python3
"""Host-side cost of one VecTrainer.step() (Python + ctypes + HIP launch calls) vs
the GPU time per step: if the first approaches the second the GPU waits on the host."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))
import torch  # noqa: E402

from evacx.env import DeviceLayout  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402
from evacx.trainer import VecTrainer  # noqa: E402

lagged = "--strict" not in sys.argv
cfg2 = "--cfg2" in sys.argv  # 64x64, 569 people, 8 robots (BASELINE cfg2), else 128x128 / 2276 / 16
lay = DeviceLayout(build_tables(synthetic(64, 64, 8) if cfg2 else synthetic(128, 128, 16)), 569 if cfg2 else 2276)
tr = VecTrainer(lay, 4096, batch=4096, lagged_learn=lagged)
for _ in range(300):
    tr.step()
tr.sync()
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for _ in range(200):
    a = time.perf_counter()
    tr.step()
    host.append(time.perf_counter() - a)
tr.sync()
torch.cuda.synchronize()
tot = (time.perf_counter() - t0) / 200
host.sort()
print(f"cfg2={cfg2} lagged={lagged} host per step: median {1e6 * host[100]:.0f} us, mean {1e6 * sum(host) / 200:.0f} us; "
      f"wall per step {1e6 * tot:.0f} us")
