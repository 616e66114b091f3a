#!/usr/bin/env python3
"""Diagnostic: phase timeline of qact3_kernel from the -DEVX_ACT_STAMPS build
(EVACX_LIB=libevacx_actst.so): wave 0's s_memtime at the phase boundaries of every workgroup.
Prints median cycles per phase and how workgroup lifetimes overlap. Never quote wall time from it."""
import ctypes as C
import os
import subprocess
import sys

os.environ.setdefault("EVACX_LIB", "libevacx_actst.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from evacx import _lib  # noqa: E402
from evacx.env import DeviceLayout, VecEnv  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402
from evacx.qnet import DROPOUT_P, Learner  # noqa: E402

frac = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
rows = 8192 * 128
E, R = 4096, 16
lay = DeviceLayout(build_tables(synthetic(128, 128, R)), 2276)
env = VecEnv(lay, E)
env.seed([1 + i for i in range(E)])
env.reset()
for _ in range(100):
    env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32))
obs = env.obs.view(-1, 8).repeat(rows // (E * R), 1).contiguous()
lr = Learner(kind="mlp", precision="f32", seed=1)
c = lay.c
lr.fast.attach_static(c, c.L, c.W, c.t_max, x_range=(c.rx_lo, c.rx_hi))
nt = int(rows * frac) // 128 * 128
obs[:nt, 6] = int(c.t_max)
act = torch.empty(rows, dtype=torch.int32, device="cuda")
for i in range(3):
    lr.fast.act(lay.c, obs.view(-1), rows, drop=(1, i, DROPOUT_P), actions=act, epsilon=0.1)
torch.cuda.synchronize()
NST = 12
buf = np.zeros(8192 * NST, np.int64)
L = _lib.lib()
L.evx_diag_act_stamps.argtypes = [C.c_void_p, C.c_int32]
n = L.evx_diag_act_stamps(buf.ctypes.data, buf.size)
assert n > 0, n
st = buf.reshape(8192, NST)
names = ["setup (W3, obs, table sync)", "h0 fc1 (table loads + occ MFMA)", "h0 epilogue -> LDS", "h0 barrier",
         "h0 fc2", "h1 barrier+fc1", "h1 epilogue", "h1 barrier", "h1 fc2", "H2 epilogue + barrier", "fc3 + eps"]
d = np.diff(st, axis=1)
tot = st[:, 11] - st[:, 0]
print(f"table frac {frac}: workgroup lifetime median {np.median(tot):.0f} cycles, mean {tot.mean():.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:34s} median {np.median(d[:, i]):8.0f}  mean {d[:, i].mean():8.0f}  share {d[:, i].sum() / tot.sum():6.1%}")
span = st[:, 11].max() - st[:, 0].min()
print(f"launch span {span} cycles; sum of lifetimes / span = {tot.sum() / span:.1f} workgroups in flight (256 CUs)")
