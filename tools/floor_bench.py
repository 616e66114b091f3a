"""Device floor-field throughput (evx_floor_field): layouts per second for batches of
random mazes, LDS path (130 x 130) and global path (258 x 258), with relaxation passes."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from evacx.floor import floor_fields  # noqa: E402
from test_floor_gpu import _mazes  # noqa: E402

for GX, n in [(130, 512), (258, 256)]:
    v, s, p = _mazes(n, GX, GX, seed=1)
    vt, st, pt = (torch.from_numpy(a).cuda() for a in (v, s, p))
    passes = torch.zeros(n, dtype=torch.int32, device="cuda")
    out = floor_fields(vt, st, pt, passes=passes)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        floor_fields(vt, st, pt, out=out, passes=passes)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 3
    pc = passes.cpu().numpy()
    print(f"floor {GX}x{GX} n={n}: {ms:8.2f} ms/launch  {n / ms * 1e3:9.0f} layouts/s  passes mean {pc.mean():.0f} max {pc.max()}")
    if GX == 130:
        from oracle import oracle as orc
        t0 = time.perf_counter()
        orc.floor_field(v[0], s[0], p[0])
        print(f"  host heapq (the reference's algorithm, 1 core): {(time.perf_counter() - t0) * 1e3:.1f} ms/layout")
