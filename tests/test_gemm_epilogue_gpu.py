"""GPU numerics of evx_gemm's split-K paths (round 2) against a plain PyTorch fp32/f64 reference:

* a long-K GEMM with an epilogue (bias, ReLU, dropout keep-mask with its scale, ReLU-backward gate)
  is split over K (each slice stores its raw partial into the caller's workspace) and
  splitk_reduce_kernel adds the slices in slice order and applies the epilogue -- the conv
  Q-net's fc1 shape (K = 15 488) at learn (32 tiles) and act (256 tiles) batches, and the same
  shapes with one tile row; bit-identical across calls (round 3: the slices were f32 atomics,
  so the conv act's Q-values could differ between runs with the same seed -- ADVICE r2);
  the same GEMM with no workspace runs in one pass (within tolerance of the split one);
* the same GEMM without an epilogue (weight-gradient shape), and with ACCUM;
* evx_colsum (bias gradients) in 64-row chunks with a per-column LDS-tree total: vs torch f64 and
  bit-identical across repeated calls (fixed summation order).

Tolerance: x3 products (bf16 hi/lo pairs, ~2^-17 relative per product, f32 accumulation in
another order than torch's) rtol 2e-4 of the output scale; colsum rtol 1e-5 (f32 sums)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("M,N,K,flags", [
    (1024, 512, 15488, "bias relu mask"),   # conv fc1, learn batch: 32 tiles -> 16 K slices
    (8192, 512, 15488, "bias relu mask"),   # conv fc1, act batch: 256 tiles -> 4 K slices
    (96, 256, 8192, "bias relu gate"),      # ragged M, gate epilogue
    (130, 200, 5000, "bias"),               # ragged M, N and K
    (512, 640, 32768, ""),                  # no epilogue (dW shape)
    (256, 300, 20000, "accum"),             # C += A B^T, split
])
def test_split_k_epilogue_matches_torch(M, N, K, flags):
    _need_gpu()
    from evacx.qnet import gemm
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.rand(M, K, device="cuda", generator=g) - 0.5
    W = (torch.rand(N, K, device="cuda", generator=g) - 0.5) * 0.05
    bias = (torch.rand(N, device="cuda", generator=g) - 0.5) if "bias" in flags else None
    mask = (torch.rand(M, N, device="cuda", generator=g) < 0.8).to(torch.uint8) if "mask" in flags else None
    gate = (torch.rand(M, N, device="cuda", generator=g) - 0.3) if "gate" in flags else None
    from evacx.qnet import _Workspace, evx_gemm_desc, qlib
    import ctypes as C_
    d = evx_gemm_desc(M=M, N=N, K=K, precision=2, flags=(1 if "relu" in flags else 0) | (2 if "accum" in flags else 0),
                      bias=1 if bias is not None else None, mask=1 if mask is not None else None,
                      gate=1 if gate is not None else None)
    need = int(qlib().evx_gemm_ws_elems(C_.byref(d)))
    assert need >= 2 * M * N, need  # these shapes split
    C0 = torch.rand(M, N, device="cuda", generator=g) if "accum" in flags else None
    outs = []
    for ws in (_Workspace(), _Workspace(), None):
        C = C0.clone() if C0 is not None else torch.full((M, N), float("nan"), device="cuda")
        gemm(M, N, K, A, K, 1, W, 1, K, C, N, "x3", bias=bias, relu="relu" in flags, mask=mask, ldm=N,
             mask_scale=1.25, gate=gate, ldg=N, accumulate="accum" in flags, ws=ws)
        outs.append(C)
    C, C2, C1 = outs
    torch.cuda.synchronize()
    assert torch.equal(C, C2)  # split-K in a fixed slice order: the same bits on every call
    ref = A.double() @ W.double().t()
    if bias is not None:
        ref = ref + bias.double()
    if "relu" in flags:
        ref = torch.relu(ref)
    if mask is not None:
        ref = torch.where(mask.bool(), ref * 1.25, torch.zeros_like(ref))
    if gate is not None:
        ref = torch.where(gate > 0, ref, torch.zeros_like(ref))
    if C0 is not None:
        ref = ref + C0.double()
    assert torch.isfinite(C).all()
    scale = ref.abs().max().item()
    for got in (C, C1):  # split and one-pass
        err = (got.double() - ref).abs().max().item()
        assert err <= 2e-4 * scale, (err, scale)
    if mask is not None:  # dropped elements are exactly 0
        assert (C[~mask.bool()] == 0).all()


@pytest.mark.parametrize("M,N", [(1, 5), (1000, 37), (123904, 32), (32768, 512)])
def test_colsum_chunked_tree(M, N):
    _need_gpu()
    from evacx.qnet import colsum
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    X = torch.rand(M, N, device="cuda", generator=g) - 0.5
    scratch = torch.empty(((M + 63) // 64) * max(N, 128), device="cuda")
    out1 = torch.empty(N, device="cuda")
    out2 = torch.empty(N, device="cuda")
    colsum(X, M, N, out1, scratch)
    colsum(X, M, N, out2, scratch)
    torch.cuda.synchronize()
    ref = X.double().sum(0)
    assert torch.equal(out1, out2)  # fixed order: deterministic
    assert (out1.double() - ref).abs().max().item() <= 1e-5 * max(1.0, X.abs().sum(0).max().item())
