#!/usr/bin/env python3
"""Microbenchmark of the fused bf16 MLP forward (evx_qmlp_forward) at act and learn sizes."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dqn-marl_amd"))
import torch  # noqa: E402

from evacx.env import DeviceLayout, VecEnv  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402
from evacx.qmlp import HID, K1P, MLPFast  # noqa: E402
from evacx.qnet import Learner  # noqa: E402

E, R = 4096, 16
lay = DeviceLayout(build_tables(synthetic(128, 128, R)), 2276)
env = VecEnv(lay, E)
env.seed([1 + i for i in range(E)])
env.reset()
for _ in range(3):
    env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32))
lr = Learner(kind="mlp", precision="bf16", seed=1)
fast = MLPFast(lr.online, "cuda")
n_all = E * R
h1 = torch.empty(n_all * HID, dtype=torch.int16, device="cuda")
x = torch.empty(n_all * K1P, dtype=torch.int16, device="cuda")
h2 = torch.empty(n_all, 256, device="cuda")
q = torch.empty(n_all, 5, device="cuda")
act = torch.empty(n_all, dtype=torch.int32, device="cuda")
flops_row = 2 * (726 * 512 + 512 * 256 + 256 * 5)
for _ in range(3):
    fast.act(lay.c, env.obs, n_all, drop=(1, 2, 0.2), actions=act, epsilon=0.1)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    fast.act(lay.c, env.obs, n_all, drop=(1, 2, 0.2), actions=act, epsilon=0.1)
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) / 20 * 1e3
print(f"{'fused act (qact_kernel)':26s} n={n_all:6d}: {us:8.1f} us  {flops_row * n_all / us / 1e6:7.1f} TF/s (whole MLP flops)")
# fast path: every env past the fire's last step (fc1 from the per-centre table)
obs_late = env.obs.view(-1, 8).clone()
obs_late[:, 6] = lay.c.t_max
fast.attach_static(lay.c, lay.c.L, lay.c.W, lay.c.t_max)
for _ in range(3):
    fast.act(lay.c, obs_late, n_all, drop=(1, 2, 0.2), actions=act, epsilon=0.1)
a.record()
for _ in range(20):
    fast.act(lay.c, obs_late, n_all, drop=(1, 2, 0.2), actions=act, epsilon=0.1)
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) / 20 * 1e3
print(f"{'fused act, static table':26s} n={n_all:6d}: {us:8.1f} us")
a.record()
for _ in range(20):
    fast._rebuild_static()
b.record()
torch.cuda.synchronize()
print(f"{'static table rebuild':26s} n={fast._static[1].shape[0]:6d}: {a.elapsed_time(b) / 20 * 1e3:8.1f} us")
fast.detach_static()
for n, kw, name in [(n_all, dict(actions=act, epsilon=0.1), "act (fc1+fc23+egreedy)"),
                    (n_all, dict(), "fc1 only"),
                    (4096, dict(x=x, h2=h2, q=q), "learn fwd (saves x,h2)"),
                    (4096, dict(q=q), "target fwd")]:
    for _ in range(3):
        fast.forward(lay.c, env.obs, n, h1, drop=(1, 2, 0.2), **kw)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    it = 20
    for _ in range(it):
        fast.forward(lay.c, env.obs, n, h1, drop=(1, 2, 0.2), **kw)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / it * 1e3
    print(f"{name:26s} n={n:6d}: {us:8.1f} us  {flops_row * n / us / 1e6:7.1f} TF/s (whole MLP flops)")
