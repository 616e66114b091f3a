import os, sys, time
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "dqn-marl_amd"))
import torch
from evacx.env import DeviceLayout, VecEnv
from evacx.layout import build_tables, synthetic
E = 4096
lay = DeviceLayout(build_tables(synthetic(128, 128, 16)), 2276)
env = VecEnv(lay, E)
env.seed([1234 + i for i in range(E)])
env.reset()
torch.cuda.synchronize()
for n in [1, 8, 64, 4096]:
    m = torch.zeros(E, dtype=torch.uint8, device="cuda"); m[:n] = 1
    env.reset(mask=m); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        env.reset(mask=m)
    b.record(); torch.cuda.synchronize()
    print(f"reset of {n} envs: {a.elapsed_time(b) / 5 * 1e3:.1f} us")
vb = lay.tables.valid
print("valid fraction interior", vb[1:-1, 1:-1].mean())
