#!/usr/bin/env python3
"""Microbenchmark of the f32-accurate (x3) fused act (evx_qmlp_act -> qact3_kernel) on
observations of a stepped 128x128 env batch, tiled to --rows rows; prints us per act and the
bf16-MFMA rate of its products (fc1: 640 hi*hi + 512 hi*lo K, fc2: 3 x 512 K)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dqn-marl_amd"))
import torch  # noqa: E402

from evacx.env import DeviceLayout, VecEnv  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402
from evacx.qnet import DROPOUT_P, Learner  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1 << 19)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--table-frac", type=float, default=0.0,
                help="fraction of rows (the first ones) at the fire's last step, through the act table "
                     "(attach_static over Map.robot_range, as the trainer)")
ap.add_argument("--order", choices=["env", "centre", "shuffle", "robot", "pair"], default="env",
                help="row order: env (the envs' own), centre (sorted by window centre: rows sharing a table row "
                     "adjacent), shuffle (random), robot (robot-major: every env's robot 0, then robot 1, ...)")
ap.add_argument("--drop-p", type=float, default=DROPOUT_P, help="dropout p of the act (0: no dropout epilogue)")
ap.add_argument("--kernel64", action="store_true", help="the 64-row kernel only (evx_qmlp_act64)")
ap.add_argument("--no-ws", action="store_true", help="no act workspace (the fallback kernel re-checks every row)")
args = ap.parse_args()
E, R = 4096, 16
lay = DeviceLayout(build_tables(synthetic(128, 128, R)), 2276)
env = VecEnv(lay, E)
env.seed([1 + i for i in range(E)])
env.reset()
for _ in range(200):
    env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32))
obs = env.obs.view(-1, 8)
reps = (args.rows + obs.shape[0] - 1) // obs.shape[0]
obs = obs.repeat(reps, 1)[:args.rows].contiguous()
lr = Learner(kind="mlp", precision="f32", seed=1)
if args.table_frac > 0:
    c = lay.c
    lr.fast.attach_static(c, c.L, c.W, c.t_max, x_range=(c.rx_lo, c.rx_hi))
    nt = int(args.rows * args.table_frac) // 128 * 128
    obs[:nt, 6] = int(c.t_max)
if args.order == "centre":
    obs = obs[torch.argsort(obs[:, 4].long() * 4096 + obs[:, 5].long(), stable=True)].contiguous()
elif args.order == "robot":
    assert args.rows % (E * R) == 0
    obs = obs.view(-1, E, R, 8).transpose(1, 2).contiguous().view(-1, 8)
elif args.order == "pair":
    assert args.rows % (E * R) == 0
    obs = obs.view(-1, E, R // 2, 2, 8).transpose(1, 2).contiguous().view(-1, 8)
elif args.order == "shuffle":
    obs = obs[torch.randperm(obs.shape[0], device="cuda")].contiguous()
act = torch.empty(args.rows, dtype=torch.int32, device="cuda")
ws = None
if not args.no_ws:
    from evacx.qmlp import act_ws_ints
    ws = torch.zeros(act_ws_ints(args.rows), dtype=torch.int32, device="cuda")
for i in range(3):
    lr.fast.act(lay.c, obs.view(-1), args.rows, drop=(1, i, args.drop_p), actions=act, epsilon=0.1,
                kernel64=args.kernel64, ws=ws)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(args.iters):
    lr.fast.act(lay.c, obs.view(-1), args.rows, drop=(1, i, args.drop_p), actions=act, epsilon=0.1,
                kernel64=args.kernel64, ws=ws)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / args.iters * 1e3
# bf16 MFMA products per row: the table path's fc1 occupancy columns (128 K, hi + lo), else the full
# fc1 (640 hi*hi + 512 hi*lo K); fc2 3 x 512 K; fc3 (5 rows padded to 32) 3 x 256 K
tf = args.table_frac
fc1 = tf * 512 * 128 * 2 + (1 - tf) * 512 * (640 + 512)
fl = args.rows * 2 * (fc1 + 256 * 512 * 3 + 32 * 256 * 3)
print(f"rows {args.rows}{' (64-row kernel)' if args.kernel64 else ''}: {us:.1f} us per act, {fl / us / 1e6:.0f} TF/s "
      f"of bf16 MFMA products ({fl / us / 1e6 / 2500:.1%} of 2.5 PF)")
