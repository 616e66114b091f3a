#!/usr/bin/env python3
"""Microbenchmark of the x3 learn chain (Learner.learn_obs, the trainer's learn step without the
replay sample) at a bench batch: compact observations of a 128x128 R16 env; prints the mean
time per learn step from HIP events (run under rocprofv3 for per-kernel times / counters).
Usage: learn_bench.py [B] [iters] [table]; table: both nets get their act tables and the
observations sit at the layout's last fire step, as in VecTrainer's stationary phase."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))

import torch  # noqa: E402

from evacx.env import DeviceLayout, VecEnv  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402
from evacx.qnet import Learner  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    R = 16
    E = max(2 * B // R, 64)
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), 2276)
    env = VecEnv(lay, E)
    env.seed([1 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(20):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    lr = Learner(kind="mlp", precision="f32", seed=1, lr=1e-4)
    obs = env.obs.view(-1, 8)
    if len(sys.argv) > 3 and sys.argv[3] == "table":
        c = lay.c
        xr = (max(c.rx_lo, 0), min(c.rx_hi, c.L + 1))
        lr.fast.attach_static(c, c.L, c.W, c.t_max, x_range=xr)
        lr.fast_t.attach_static(c, c.L, c.W, c.t_max, x_range=xr)
        obs = obs.clone()
        obs[:, 6] = int(c.t_max)
    perm = torch.randperm(E * R, device="cuda", generator=g)
    s, s2 = obs[perm[:B]].contiguous().view(-1), obs[perm[B:2 * B]].contiguous().view(-1)
    a = torch.randint(0, 5, (B,), device="cuda", dtype=torch.int32, generator=g)
    r = torch.randn(B, device="cuda", generator=g) * 10
    d = (torch.rand(B, device="cuda", generator=g) < 0.05).to(torch.uint8)
    for _ in range(3):
        lr.learn_obs(lay.c, s, a, r, d, s2, B)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(iters):
        lr.learn_obs(lay.c, s, a, r, d, s2, B)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / iters
    print(f"learn B={B}: {ms * 1e3:.1f} us per step, loss {lr.loss.item():.4g}")


if __name__ == "__main__":
    main()
