#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of env_step_kernel from in-kernel s_memtime
stamps (evx_step_out.stamps). Shares only -- never quote this run's wall time."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from evacx.env import DeviceLayout, VecEnv, _ptr  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402

# stamp slots written by env_step_kernel (one wave per env)
SLOTS = [(0, "start"), (1, "load+robots+near"), (2, "rows(health+plan)"), (3, "contested+mt_store"),
         (4, "execute+rmap"), (5, "reward rows"), (6, "reward formula"), (8, "obs")]

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--grid", type=int, default=128)
ap.add_argument("--people", type=int, default=2276)
ap.add_argument("--robots", type=int, default=16)
ap.add_argument("--warmup", type=int, default=1300)
ap.add_argument("--stagger", type=int, default=1200)
ap.add_argument("--no-order", action="store_true", help="identity dispatch order (no heavy workgroups)")
ap.add_argument("--reset-all", action="store_true",
                help="after the warm-up reset every env (the bench's start-of-episode phase: fire kept)")
args = ap.parse_args()
E, R = args.envs, args.robots
spec = synthetic(args.grid, args.grid, R)
lay = DeviceLayout(build_tables(spec), args.people)
env = VecEnv(lay, E)
env.seed([1234 + i for i in range(E)])
env.reset()
acts = torch.randint(0, 5, (args.warmup + 3, E * R), device="cuda", dtype=torch.int32)
gid = torch.arange(E, device="cuda")
for i in range(args.warmup):
    env.step(acts[i], order=not args.no_order)
    m = env.done.bool()
    if args.stagger and i < args.stagger:
        m = m | (gid % args.stagger == i)
    env.reset(mask=m)
if args.reset_all:
    env.reset()
stamps = torch.zeros(E * 48, dtype=torch.int64, device="cuda")
env.out.stamps = _ptr(stamps)
for i in range(3):
    env.step(acts[args.warmup + i], order=not args.no_order)
torch.cuda.synchronize()
s = stamps.view(E, 48).cpu().numpy()
cols = [c for c, _ in SLOTS]
d = np.diff(s[:, cols], axis=1)
tot = s[:, cols[-1]] - s[:, 0]
order = np.argsort(tot)
top = order[-max(1, E // 100):]  # the slowest 1 % of envs
print(f"envs={E} cycles/env-step (wave lifetime, shader cycles): median {np.median(tot):.0f}  p90 "
      f"{np.percentile(tot, 90):.0f}  p99 {np.percentile(tot, 99):.0f}  max {tot.max():.0f}")
print(f"  {'phase':28s} {'median':>9s} {'mean':>9s} {'share':>7s} {'slowest1%':>10s}")
for i, (_, n) in enumerate(SLOTS[1:]):
    print(f"  {n:28s} {np.median(d[:, i]):9.0f} {d[:, i].mean():9.0f} {d[:, i].sum() / tot.sum():7.1%}"
          f" {d[top, i].mean():10.0f}")
if not s[:, 16:30].any() and s[:, 15].any():  # normal build: stamps around the observation writes
    o1, o2 = s[:, 15] - s[:, 6], s[:, 7] - s[:, 15]
    print(f"  obs: before the writes median {np.median(o1):.0f}, writes {np.median(o2):.0f}, after {np.median(s[:, 8] - s[:, 7]):.0f}")
print("py words/step median", np.median(s[:, 12]), " np words/step median", np.median(s[:, 13]),
      " contested movers median/max", np.median(s[:, 14]), s[:, 14].max(), " planners median/max",
      np.median(s[:, 11]), s[:, 11].max())
print(f"  slowest 1%: planners {s[top, 11].mean():.0f}, contested {s[top, 14].mean():.0f}")
life = s[:, 10] - s[:, 9]  # s_memrealtime: constant 100 MHz on every XCD
span = s[:, 10].max() - s[:, 9].min()
# resident envs per CU over the launch (10-us buckets): ramp, plateau, tail
t0r = s[:, 9].min()
nb = int(span // 1000) + 1
occ = np.zeros(nb)
for st_, en_ in zip((s[:, 9] - t0r) / 1000.0, (s[:, 10] - t0r) / 1000.0):
    a_, b_ = int(st_), int(en_)
    occ[a_:b_ + 1] += 1
print("resident envs per CU by 10-us bucket:", " ".join(f"{x / 256:.1f}" for x in occ))
print(f"launch span {span / 100:.1f} us; median env lifetime {np.median(life) / 100:.1f} us, max {life.max() / 100:.1f} us; "
      f"mean concurrent envs {life.sum() / span:.0f} ({life.sum() / span / 256:.2f} per CU)")
PROF = [(16, "rows: np draws+health"), (17, "rows: health sum"), (18, "rows: plan+queue+stores"),
        (19, "rows: score batches"), (20, "rows: loop top+selects"), (21, "reward: per group"),
        (22, "reward: leaves"), (23, "reward: loop top"), (24, "contested: list"), (25, "contested: groups"),
        (26, "contested: mt_store+clear"), (27, "load: mt+rmap+robots"), (28, "load: not-dead list"),
        (29, "load: near map+sync"), (30, "score: floor loads"), (31, "score: mt ensure"),
        (15, "score: scoring"), (7, "score: tail"), (32, "groups: sort"), (33, "groups: heads+sort"),
        (34, "groups: pass1 (positions)"), (35, "groups: pass2 (shuffles)")]
if s[:, 16:30].any():
    print("sub-phase cycle accumulators (EVX_PROFILE build):        median   slowest1%")
    for c, n in PROF:
        print(f"  {n:28s} {np.median(s[:, c]):9.0f} {s[top, c].mean():10.0f}")
if s[:, 46].any():
    nw, ng = s[:, 46] >> 16, s[:, 46] & 0xFFFF
    print(f"contested pass 1: windows built median {np.median(nw):.0f} slowest1% {nw[top].mean():.1f}; groups median "
          f"{np.median(ng):.0f} slowest1% {ng[top].mean():.1f}; window cycles slowest1% {s[top, 47].mean():.0f}")
WIDE = [(36, "wide: pass1 (np counts)"), (37, "wide: barrier+copy"), (38, "wide: np gen"), (39, "wide: pass2"),
        (40, "wide: np store"), (41, "wide: py setup"), (42, "wide: py gen"), (43, "wide: scoring"),
        (44, "wide: movers+plan+handoff"), (45, "wide: final barrier")]
if s[:, 36:46].any():
    hv = s[:, 36:46].sum(1) > 0
    tw = order[-max(1, E // 100):]
    print(f"wide rows (EVX_PROFILE build), {hv.sum()} heavy envs:   median(heavy)  slowest1%")
    for c, n in WIDE:
        print(f"  {n:28s} {np.median(s[hv, c]):9.0f} {s[tw, c].mean():10.0f}")
    t0 = s[:, 9].min()
    st_us, en_us = (s[:, 9] - t0) / 100, (s[:, 10] - t0) / 100
    for nm, m in [("wide", hv), ("single-wave", ~hv)]:
        if m.any():
            print(f"  {nm:12s} n={m.sum():5d} lifetime us median {np.median(life[m]) / 100:6.1f} max {life[m].max() / 100:6.1f}"
                  f"  start max {st_us[m].max():6.1f}  end max {en_us[m].max():6.1f}  planners median {np.median(s[m, 11]):.0f}")
    nw = ~hv
    top_single = np.argsort(life * nw)[-10:]
    print("  slowest single-wave envs: life us", (life[top_single] / 100).round(1), "planners", s[top_single, 11])
if os.environ.get("EVX_FCX_REPORT"):  # -DEVX_FCX build: first changed not-dead-list index vs the list length
    fcx, nnd = s[:, 36], s[:, 37]
    frac = np.where(fcx >= 0x7fffffff, 1.0, np.minimum(fcx, nnd) / np.maximum(nnd, 1))
    print(f"first changed index / list length: median {np.median(frac):.3f} mean {frac.mean():.3f}; "
          f"unchanged envs {np.mean(fcx >= 0x7fffffff):.3f}; list length median {np.median(nnd):.0f}")
    for q in (0.1, 0.25, 0.5, 0.75):
        print(f"  P(frac >= {q}) = {np.mean(frac >= q):.3f}")
# cycle share by planners per env-step (light envs: few planners; heavy: early in their episodes)
npl = s[:, 11]
print("cycle share by planners/env-step:")
for lo, hi in [(0, 1), (1, 8), (8, 64), (64, 256), (256, 1024), (1024, 1 << 30)]:
    m = (npl >= lo) & (npl < hi)
    print(f"  [{lo:5d},{hi:10d}) envs {m.mean():6.1%}  cycles {tot[m].sum() / tot.sum():6.1%}  mean {tot[m].mean() if m.any() else 0:9.0f}")
cnt = env.counts.view(E, 2).cpu().numpy()
print("evacuated median", np.median(cnt[:, 0]), "dead median", np.median(cnt[:, 1]))
