#!/usr/bin/env python3
"""Microbenchmark of evx_gemm on the learner's shapes (TFLOP/s, and max error vs torch fp32)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dqn-marl_amd"))
import torch  # noqa: E402

from evacx.qnet import gemm  # noqa: E402

# (name, M, N, K, A layout (sam, sak) fn, B layout fn, description)
SHAPES = [
    ("act fc1 fwd", 65536, 512, 726, "nt"),
    ("act fc2 fwd", 65536, 256, 512, "nt"),
    ("learn fc1 fwd", 4096, 512, 726, "nt"),
    ("learn dW1", 512, 726, 4096, "tn"),
    ("learn dW2", 256, 512, 4096, "tn"),
    ("learn dX2", 4096, 512, 256, "nn"),
]


def run(name, M, N, K, kind, prec, iters=20):
    if kind == "nt":   # C = A[M,K] . W[N,K]^T
        A = torch.randn(M, K, device="cuda")
        Bm = torch.randn(N, K, device="cuda") * 0.05
        args = (A, K, 1, Bm, 1, K)
        ref = lambda: A @ Bm.t()  # noqa: E731
    elif kind == "tn":  # C = dY[K,M]^T . X[K,N]
        A = torch.randn(K, M, device="cuda")
        Bm = torch.randn(K, N, device="cuda") * 0.05
        args = (A, 1, M, Bm, N, 1)
        ref = lambda: A.t() @ Bm  # noqa: E731
    else:  # nn: C = dY[M,K] . W[K,N]
        A = torch.randn(M, K, device="cuda")
        Bm = torch.randn(K, N, device="cuda") * 0.05
        args = (A, K, 1, Bm, N, 1)
        ref = lambda: A @ Bm  # noqa: E731
    C = torch.empty(M, N, device="cuda")
    gemm(M, N, K, *args, C, N, prec)
    torch.cuda.synchronize()
    R = ref()
    err = ((C - R).abs().max() / R.abs().max()).item()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        gemm(M, N, K, *args, C, N, prec)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    print(f"{name:14s} {prec:4s} M={M:6d} N={N:4d} K={K:5d}  {dt * 1e6:8.1f} us  {2 * M * N * K / dt / 1e12:7.1f} TF/s"
          f"  rel.err {err:.2e}")


if __name__ == "__main__":
    for s in SHAPES:
        for prec in ["bf16", "f32"]:
            run(*s, prec)
