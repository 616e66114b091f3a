#!/usr/bin/env python3
"""Diagnostic: slot timeline of the persistent x3 act (qact3p_kernel) from the -DEVX_ACT_STAMPS build
(EVX_LIB=.../libevacx_actst.so): wave 0's s_memtime at the slot boundaries of every tile. Prints
median cycles per phase. Never quote wall time from it (stamps cost cycles)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("EVX_LIB", os.path.join(ROOT, "dqn-marl_amd", "evacx", "libevacx_actst.so"))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from evacx import _lib  # noqa: E402
from evacx.env import DeviceLayout, VecEnv  # noqa: E402
from evacx.layout import build_tables, synthetic  # noqa: E402
from evacx.qnet import DROPOUT_P, Learner  # noqa: E402

rows = 1 << 19
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
obs[:, 6] = int(c.t_max)
act = torch.empty(rows, dtype=torch.int32, device="cuda")
for i in range(5):
    lr.fast.act(lay.c, obs.view(-1), rows, drop=(1, i, DROPOUT_P), actions=act, epsilon=0.1)
torch.cuda.synchronize()
NST, MAXIT = 16, 32
buf = np.zeros(256 * MAXIT * NST, np.int64)
L = _lib.lib()
L.evx_diag_act3p_stamps.argtypes = [C.c_void_p, C.c_int32]
n = L.evx_diag_act3p_stamps(buf.ctypes.data, buf.size)
assert n > 0, n
st = buf.reshape(256, MAXIT, NST)
ntile = rows // 128
its = (ntile + 255) // 256
st = st[:, :its].reshape(-1, NST)[:, :14]
st = st[st[:, 13] > 0]
names = ["loop top -> tile set up", "slot0 fc1(q0)", "slot0 fc2(prev q3) + epilogue(q0) + fc3 partials(prev)",
         "slot0 barrier + rows(prev)", "slot1 fc1(q1)", "slot1 fc2(q0) + epilogue(q1)", "slot1 barrier", "slot2 fc1(q2)",
         "slot2 fc2(q1) + epilogue(q2) + next rows", "slot2 barrier (and)", "slot3 fc1(q3) + next occ",
         "slot3 fc2(q2) + epilogue(q3)", "slot3 barrier"]
d = np.diff(st, axis=1)
tot = st[:, 13] - st[:, 0]
print(f"tiles {len(st)}: tile median {np.median(tot):.0f} cycles, mean {tot.mean():.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:44s} median {np.median(d[:, i]):8.0f}  mean {d[:, i].mean():8.0f}  share {d[:, i].sum() / tot.sum():6.1%}")
