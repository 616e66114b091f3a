#!/usr/bin/env python3
"""Microbenchmark of the x3 implicit-GEMM 3x3 convolutions (evx_conv3x3_gemm) at the cfg4 act's shapes:
forward of conv1/2/3 over B x 121 pixels (TFLOP/s of bf16 products, 3 per f32 MAC) and the max
relative error against torch's fp64 conv2d. Usage: python tools/conv_bench.py [B]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dqn-marl_amd"))
import torch  # noqa: E402

from evacx.qnet import CONV_FWD, conv_gemm  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
g = torch.Generator(device="cuda").manual_seed(0)
for cin, cout in [(6, 32), (32, 64), (64, 128)]:
    Mp, K9 = B * 121, cin * 9
    x = torch.rand(Mp, cin, device="cuda", generator=g)
    w = (torch.rand(cout, cin, 3, 3, device="cuda", generator=g) - 0.5) * 0.2
    b = (torch.rand(cout, device="cuda", generator=g) - 0.5) * 0.1
    y = torch.empty(Mp, cout, device="cuda")
    run = lambda: conv_gemm(CONV_FWD, Mp, cout, K9, x, w, y, cin, sbk=9, sbn=K9, bias=b, relu=True)  # noqa: E731
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 100.0
    xs = x[: 64 * 121].view(64, 11, 11, cin).permute(0, 3, 1, 2).double()
    ref = torch.relu(torch.nn.functional.conv2d(xs, w.double(), b.double(), padding=1)).permute(0, 2, 3, 1)
    err = ((y[: 64 * 121].view(64, 11, 11, cout).double() - ref).abs().max() / ref.abs().max()).item()
    tf = 2.0 * Mp * cout * K9 * 3 / (us * 1e-6) / 1e12
    print(f"conv {cin:3d}->{cout:3d}: {us:8.1f} us  {tf:7.1f} TF/s (bf16 products)  max rel err {err:.2e}", flush=True)
