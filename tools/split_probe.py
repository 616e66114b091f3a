#!/usr/bin/env python3
"""env.step split into its heavy part (evx_env_step_part 1) and the rest (part 2): how
long each takes alone and both concurrently on two streams, vs the one-launch step, on
the bench workload (cfg3 share, staggered env ages). Event timing per stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))
import torch  # noqa: E402

from evacx.env import DeviceLayout, VecEnv  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402

E, R, P = 4096, 16, 2276
lay = DeviceLayout(build_tables(synthetic(128, 128, R)), P)
env = VecEnv(lay, E, obs_buffers=2)
env.seed([1234 + i for i in range(E)])
env.reset()
g = torch.Generator(device="cuda").manual_seed(1)
gid = torch.arange(E, device="cuda")
for w in range(1300):
    env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    if w < 1200:
        env.reset(mask=(gid % 1200) == w)
torch.cuda.synchronize()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
cur = torch.cuda.current_stream()


def ev():
    return torch.cuda.Event(enable_timing=True)


res = {k: [] for k in ["one", "heavy_alone", "light_alone", "both_heavy", "both_light", "both_span"]}
for it in range(30):
    acts = torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g)
    mode = it % 3
    env.compute_order()
    H = None
    if mode == 0:
        a, b = ev(), ev()
        a.record()
        env.step(acts, order=False, auto_reset=True)
        b.record()
        torch.cuda.synchronize()
        res["one"].append(a.elapsed_time(b))
    elif mode == 1:
        a, b, c = ev(), ev(), ev()
        a.record()
        env.step(acts, order=False, auto_reset=True, part=1)
        b.record()
        env.step(acts, order=False, auto_reset=True, part=2)
        c.record()
        torch.cuda.synchronize()
        res["heavy_alone"].append(a.elapsed_time(b))
        res["light_alone"].append(b.elapsed_time(c))
    else:
        a = ev()
        a.record()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        b1, b2 = ev(), ev()
        with torch.cuda.stream(s1):
            env.step(acts, order=False, auto_reset=True, part=1)
            b1.record(s1)
        with torch.cuda.stream(s2):
            env.step(acts, order=False, auto_reset=True, part=2)
            b2.record(s2)
        cur.wait_stream(s1)
        cur.wait_stream(s2)
        torch.cuda.synchronize()
        res["both_heavy"].append(a.elapsed_time(b1))
        res["both_light"].append(a.elapsed_time(b2))
        res["both_span"].append(max(a.elapsed_time(b1), a.elapsed_time(b2)))
    if it == 29:
        print("heavy envs this step:", int(env.order[E].item()))
for k, v in res.items():
    v = sorted(v)
    print(f"{k:12s} median {v[len(v) // 2] * 1e3:7.1f} us  (n={len(v)})")
env.check_err()
