"""GPU numerics of the learner kernels (evx_gemm / td_loss / clip+Adam / conv helpers)
against a plain PyTorch fp32 reference of the same network with the same dropout masks.

Tolerances: exact-f32 MFMA path and the x3 conv path (bf16 hi/lo operand pairs, product
error ~2^-17 relative) rtol 2e-4 / atol 2e-5 (summation order differs from torch's); bf16 MFMA path rtol 3e-2 on Q-values (bf16 inputs, f32 accumulation)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def torch_forward(kind, sd, x, mask):
    """agents/dqn_agent.py:35-61 with an injected dropout keep-mask."""
    B = x.shape[0]
    if kind == "conv":
        h = x.permute(0, 3, 1, 2).contiguous()
        h = F.relu(F.conv2d(h, sd["conv1.weight"], sd["conv1.bias"], padding=1))
        h = F.relu(F.conv2d(h, sd["conv2.weight"], sd["conv2.bias"], padding=1))
        h = F.relu(F.conv2d(h, sd["conv3.weight"], sd["conv3.bias"], padding=1))
        h = h.reshape(B, -1)
    else:
        h = x.reshape(B, -1)
    h = F.relu(F.linear(h, sd["fc1.weight"], sd["fc1.bias"]))
    if mask is not None:
        h = h * mask.float() / 0.8
    h = F.relu(F.linear(h, sd["fc2.weight"], sd["fc2.bias"]))
    return F.linear(h, sd["fc3.weight"], sd["fc3.bias"])


def make_batch(B, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.rand(B, 11, 11, 6, generator=g) < 0.3).float()
    x[..., 2] = torch.rand(B, 11, 11, generator=g) * 0.8
    x2 = (torch.rand(B, 11, 11, 6, generator=g) < 0.3).float()
    a = torch.randint(0, 5, (B,), generator=g, dtype=torch.int32)
    r = torch.randn(B, generator=g) * 50
    d = (torch.rand(B, generator=g) < 0.1).to(torch.uint8)
    m1 = (torch.rand(B, 512, generator=g) >= 0.2).to(torch.uint8)
    m2 = (torch.rand(B, 512, generator=g) >= 0.2).to(torch.uint8)
    return x, x2, a, r, d, m1, m2


@pytest.mark.parametrize("kind,prec", [("mlp", "f32"), ("conv", "f32"), ("conv", "x3")])
def test_forward_f32_matches_torch(kind, prec):
    _need_gpu()
    from evacx.qnet import Learner
    lr = Learner(kind=kind, precision=prec, seed=3)
    x, _, _, _, _, m1, _ = make_batch(37, 0)
    q = lr.net.forward(x.cuda(), m1.cuda(), save=False).cpu()
    sd = {k: v.cpu() for k, v in lr.online.state_dict().items()}
    ref = torch_forward(kind, sd, x, m1)
    torch.testing.assert_close(q, ref, rtol=2e-4, atol=2e-5)


def test_forward_bf16_close_to_torch():
    _need_gpu()
    from evacx.qnet import Learner
    lr = Learner(kind="mlp", precision="bf16", seed=4)
    x, _, _, _, _, m1, _ = make_batch(300, 1)
    q = lr.net.forward(x.cuda(), m1.cuda(), save=False).cpu()
    ref = torch_forward("mlp", {k: v.cpu() for k, v in lr.online.state_dict().items()}, x, m1)
    err = (q - ref).abs().max() / ref.abs().max()
    assert err < 3e-2, err


@pytest.mark.parametrize("kind,prec", [("mlp", "f32"), ("conv", "f32"), ("conv", "x3")])
def test_learn_steps_match_torch_adam(kind, prec):
    """3 learn steps: loss, clipped grads and params vs torch (MSE, clip_grad_norm_(1.0), Adam 1e-4).
    (cfg4's batch, B = 1024: tests/test_bench_scale_gpu.py::test_conv_x3_learn_at_cfg4_batch.)"""
    _need_gpu()
    from evacx.qnet import Learner
    B = 32
    lr = Learner(kind=kind, precision=prec, seed=5, lr=1e-3)
    sd0 = {k: v.cpu().clone() for k, v in lr.online.state_dict().items()}
    params = {k: torch.nn.Parameter(v.clone()) for k, v in sd0.items()}
    tgt = {k: v.clone() for k, v in sd0.items()}
    opt = torch.optim.Adam(params.values(), lr=1e-3)
    for it in range(3):
        if it > 0:  # each step is compared from the same state (params + Adam moments)
            lr.online.load_state_dict({k: p.detach() for k, p in params.items()})
            for key, buf in (("exp_avg", lr.m), ("exp_avg_sq", lr.v)):
                buf.copy_(torch.cat([opt.state[p][key].reshape(-1) for p in params.values()]).cuda())
        x, x2, a, r, d, m1, m2 = make_batch(B, 10 + it)
        loss = lr.learn(x.cuda(), a.cuda(), r.float().cuda(), d.cuda(), x2.cuda(), m1.cuda(), m2.cuda())
        q = torch_forward(kind, params, x, m1).gather(1, a.long().unsqueeze(1))
        with torch.no_grad():
            nq = torch_forward(kind, tgt, x2, m2).max(1)[0]
            y = r.float() + 0.99 * nq * (~d.bool())
        ref_loss = F.mse_loss(q.squeeze(), y)
        opt.zero_grad()
        ref_loss.backward()
        gnorm = torch.nn.utils.clip_grad_norm_(params.values(), 1.0)
        grads_ref = {k: p.grad.clone() for k, p in params.items()}
        flipped = _relu_flips(lr, params, x) if prec == "x3" else set()  # params before the step
        opt.step()
        assert abs(loss.item() - ref_loss.item()) <= 2e-4 * abs(ref_loss.item()) + 1e-5
        assert abs(lr.norm.item() - gnorm.item()) <= 2e-4 * gnorm.item() + 1e-6
        for k in params:
            # x3: a product is ~2^-17 off (bf16 hi + lo pairs, lo*lo dropped), so a gradient element is
            # off by ~2^-17 of its sum of |products|, not of its value: atol scales with the tensor
            # (1e-3 of its max |grad|; the reference's own CUDA conv runs TF32, 2^-11 per product).
            # A conv pre-activation within that error of 0 can take the other relu branch than
            # torch's (_relu_flips checks it is one): that layer's and the lower layers' gradients
            # then differ by the flipped pixel's share -- bar 5e-2 of max |grad| for those.
            atol = 2e-6
            if prec == "x3":
                atol = (5e-2 if k.split(".")[0] in flipped else 1e-3) * grads_ref[k].abs().max().item()
            torch.testing.assert_close(lr.grads[k].cpu(), grads_ref[k], rtol=2e-3, atol=atol)
            # Adam divides by sqrt(v): for near-zero gradients a last-bit grad difference moves
            # that element's update by a visible fraction of lr. Bar: at most 1e-4 of the
            # elements beyond 1e-5 (1% of a step, lr = 1e-3), none beyond one full step; x3 (its
            # gradients ~2^-17 off per product, split-K atomics) 2e-3 of them.
            diff = (lr.online[k].cpu() - params[k].detach()).abs()
            bar = 2e-3 if prec == "x3" else 1e-4
            if k.split(".")[0] not in flipped:
                assert (diff > 1e-5).float().mean().item() <= bar, (k, diff.max().item())
            # one Adam step moves an element by at most lr (1-b1)/sqrt(1-b2) ~ 3.2 lr: below a relu
            # flip a near-zero gradient may change sign, so there the bar is two such steps
            assert diff.max().item() <= (6.4e-3 if k.split(".")[0] in flipped else 1e-3), (k, diff.max().item())


def _relu_flips(lr, params, x):
    """Conv layers whose relu took the other branch than torch's at some pixel, and every layer
    below one (their gradients flow through it). Each flipped pre-activation must be within the
    x3 rounding of 0: |z| <= 1e-4 of the layer's max |z|."""
    B = x.shape[0]
    h = x.permute(0, 3, 1, 2).contiguous()
    names = ("conv1", "conv2", "conv3")
    out = set()
    for li, c in enumerate(names):
        z = F.conv2d(h, params[c + ".weight"].detach(), params[c + ".bias"].detach(), padding=1)
        yg = lr.net.saved["ys"][li].cpu().reshape(B, 11, 11, -1).permute(0, 3, 1, 2)
        bad = (z > 0) != (yg > 0)
        if bad.any():
            assert z[bad].abs().max().item() <= 1e-4 * z.abs().max().item(), (c, z[bad].abs().max().item())
            out.update(names[:li + 1])
        h = F.relu(z)
    return out


def test_act_argmax_and_epsilon():
    _need_gpu()
    from evacx import qnet
    Q = torch.tensor([[0, 1, 3, 3, 2], [5, 5, 5, 5, 5], [-1, -2, -3, -4, -0.5]], dtype=torch.float32).cuda()
    out = torch.zeros(3, dtype=torch.int32, device="cuda")
    qnet.qcheck(qnet.qlib().evx_act(Q.data_ptr(), 3, 5, 0.0, 1, 0, out.data_ptr(), qnet._stream()), "act")
    assert out.cpu().tolist() == [2, 0, 4]  # first maximum, as np.argmax
    Qb = torch.zeros(100000, 5, device="cuda")
    Qb[:, 3] = 1
    ob = torch.zeros(100000, dtype=torch.int32, device="cuda")
    qnet.qcheck(qnet.qlib().evx_act(Qb.data_ptr(), 100000, 5, 0.25, 7, 0, ob.data_ptr(), qnet._stream()), "act")
    frac = (ob != 3).float().mean().item()
    assert abs(frac - 0.25 * 0.8) < 0.01  # random action is 3 one time in five


def test_dropout_mask_rate():
    _need_gpu()
    from evacx import qnet
    m = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    qnet.qcheck(qnet.qlib().evx_dropout_mask(m.data_ptr(), m.numel(), 0.2, 11, 0, qnet._stream()), "mask")
    assert abs(m.float().mean().item() - 0.8) < 0.003


@pytest.mark.parametrize("cin,cout,B", [(6, 32, 5), (32, 64, 3), (64, 128, 2), (5, 7, 4)])
def test_conv3x3_implicit_gemm_vs_torch(cin, cout, B):
    """evx_conv3x3_gemm forward / dX (with the ReLU gate of the layer below) / dW against torch's
    conv2d and autograd in float64 (the same 3x3 padding-1 conv as DQNNetwork's, dqn_agent.py:22-24).
    x3 precision: error ~2^-17 of the sum of |products| -> atol scales with the tensor."""
    _need_gpu()
    from evacx import qnet
    g = torch.Generator().manual_seed(cin * 100 + cout)
    x = torch.randn(B, 11, 11, cin, generator=g)           # pixel-major = NHWC
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.2
    bias = torch.randn(cout, generator=g) * 0.1
    dy = torch.randn(B, 11, 11, cout, generator=g)
    below = torch.randn(B, 11, 11, cin, generator=g)        # the layer below's relu output (gate)
    Mp, K9 = B * 121, cin * 9
    xd, wd, bd, dyd, gd = (t.cuda().contiguous() for t in (x, w, bias, dy, below))
    y = torch.zeros(Mp, cout, device="cuda")
    qnet.conv_gemm(qnet.CONV_FWD, Mp, cout, K9, xd, wd, y, cin, sbk=9, sbn=K9, bias=bd, relu=True)
    dx = torch.zeros(Mp, cin, device="cuda")
    qnet.conv_gemm(qnet.CONV_DX, Mp, cin, cout * 9, dyd, wd, dx, cout, sbk=K9, sbn=9, gate=gd, ldg=cin)
    dw = torch.full((cout, K9), 7.0, device="cuda")        # overwritten (split-K zeroes it first)
    qnet.conv_gemm(qnet.CONV_DW, cout, K9, Mp, dyd, xd, dw, cin, sam=1, sak=cout)
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.double().requires_grad_(True)
    z = F.conv2d(xr, wr, bias.double(), padding=1)
    yref = F.relu(z).permute(0, 2, 3, 1).reshape(Mp, cout)
    z.backward(dy.double().permute(0, 3, 1, 2))
    dxref = (xr.grad.permute(0, 2, 3, 1) * (below.double() > 0)).reshape(Mp, cin)
    dwref = wr.grad.reshape(cout, K9)
    for got, ref in ((y, yref), (dx, dxref), (dw, dwref)):
        ref = ref.detach().float()
        torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=2e-5 * ref.abs().max().item())


@pytest.mark.parametrize("cin,cout,B,split", [(32, 64, 16, False), (64, 128, 16, False), (64, 128, 64, True),
                                              (32, 64, 40, True)])
def test_conv3x3_dw_tn_kernel_vs_torch(cin, cout, B, split):
    """The conv weight gradient on the k-major x3 kernel (tn3_kernel: channels a multiple of 4,
    K = B*121 >= 256), one K pass or split into the workspace: against torch autograd in float64."""
    _need_gpu()
    from evacx import qnet
    g = torch.Generator().manual_seed(cin * 7 + B)
    x = torch.randn(B, 11, 11, cin, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.2
    dy = torch.randn(B, 11, 11, cout, generator=g)
    Mp, K9 = B * 121, cin * 9
    xd, dyd = x.cuda().contiguous(), dy.cuda().contiguous()
    dw = torch.full((cout, K9), 7.0, device="cuda")
    ws = torch.zeros(1 << 24, device="cuda") if split else None
    qnet.conv_gemm(qnet.CONV_DW, cout, K9, Mp, dyd, xd, dw, cin, sam=1, sak=cout, ws=ws)
    xr = x.double().permute(0, 3, 1, 2)
    wr = w.double().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(dy.double().permute(0, 3, 1, 2))
    ref = wr.grad.reshape(cout, K9).float()
    torch.testing.assert_close(dw.cpu(), ref, rtol=1e-4, atol=2e-5 * ref.abs().max().item())


@pytest.mark.parametrize("M,N,K,split", [(512, 1000, 1500, False), (256, 512, 4100, True), (64, 96, 3000, True)])
def test_gemm_x3_k_major_operands_vs_float64(M, N, K, split):
    """evx_gemm x3 with A[k][m] (sam 1) and B[k][n] (sbn 1) -- the fc layers' weight gradients
    dW = dZ^T X on tn3_kernel (ragged M / N / K tiles, one pass or split-K) -- against float64."""
    _need_gpu()
    from evacx import qnet
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(K, M, generator=g)
    Bm = torch.randn(K, N, generator=g)
    C = torch.full((M, N), 3.0, device="cuda")
    ws = torch.zeros(1 << 24, device="cuda") if split else None
    qnet.gemm(M, N, K, A.cuda(), 1, M, Bm.cuda(), N, 1, C, N, "x3", ws=ws)
    ref = (A.double().t() @ Bm.double()).float()
    torch.testing.assert_close(C.cpu(), ref, rtol=1e-4, atol=2e-5 * ref.abs().max().item())


@pytest.mark.parametrize("M,N,K,epi", [(1024, 1000, 512, "gate"), (300, 512, 256, "mask_gate"), (256, 640, 1000, "bias_relu"),
                                       (96, 128, 4096, "accum")])
def test_gemm_x3_k_contiguous_a_n_contiguous_b_vs_float64(M, N, K, epi):
    """evx_gemm x3 with A[m][k] (sak 1) and B[k][n] (sbn 1) -- the fc layers' activation gradients
    dX = dY W (tn3_kernel's k-contiguous A) -- with evx_gemm's epilogues (bias, ReLU, dropout mask x
    scale, ReLU gate, accumulate), against float64."""
    _need_gpu()
    from evacx import qnet
    g = torch.Generator().manual_seed(M * 3 + N + K)
    A = torch.randn(M, K, generator=g)
    Bm = torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    mask = (torch.rand(M, N, generator=g) < 0.8).to(torch.uint8)
    gate = torch.randn(M, N, generator=g)
    ref = A.double() @ Bm.double()
    kw = {}
    if "bias" in epi:
        kw["bias"] = bias.cuda()
        ref = ref + bias.double()
    if "relu" in epi:
        kw["relu"] = True
        ref = ref.clamp_min(0)
    if "mask" in epi:
        kw.update(mask=mask.cuda(), ldm=N, mask_scale=1.25)
        ref = torch.where(mask.bool(), ref * 1.25, torch.zeros_like(ref))
    if "gate" in epi:
        kw.update(gate=gate.cuda(), ldg=N)
        ref = torch.where(gate > 0, ref, torch.zeros_like(ref))
    if epi == "accum":
        kw["accumulate"] = True
        ref = ref + C0.double()
    C = C0.clone().cuda()
    qnet.gemm(M, N, K, A.cuda(), K, 1, Bm.cuda(), N, 1, C, N, "x3", **kw)
    ref = ref.float()
    torch.testing.assert_close(C.cpu(), ref, rtol=1e-4, atol=2e-5 * ref.abs().max().item())


@pytest.mark.parametrize("M,N,K,split", [(8192, 512, 15488, False), (300, 200, 1000, False), (256, 512, 6144, True)])
def test_gemm_x3_split_ab_vs_float64(M, N, K, split):
    """evx_gemm with EVX_GEMM_SPLIT_AB (A [2][M][K], B [2][N][K] bf16 hi / lo planes, k-contiguous: the
    conv net's fc1 forward) with bias and ReLU, against float64 of the unsplit values;
    cfg4's act shape (8192 x 512 x 15488), ragged tiles, and split-K."""
    _need_gpu()
    from evacx import qnet
    g = torch.Generator().manual_seed(M + 7 * N + K)
    A = torch.randn(M, K, generator=g)
    Bm = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g)

    def planes(x):
        hi = x.to(torch.bfloat16)
        lo = (x - hi.float()).to(torch.bfloat16)
        return torch.stack([hi, lo]).view(torch.int16).cuda().contiguous()
    C = torch.full((M, N), 5.0, device="cuda")
    ws = torch.zeros(1 << 24, device="cuda") if split else None
    qnet.gemm(M, N, K, planes(A), K, 1, planes(Bm), 1, K, C, N, "x3", bias=bias.cuda(), relu=True, ws=ws, split_ab=True)
    ref = (A.double() @ Bm.double().t() + bias.double()).clamp_min(0).float()
    torch.testing.assert_close(C.cpu(), ref, rtol=1e-4, atol=2e-5 * ref.abs().max().item())


def test_conv_x3_act_and_learn_are_deterministic():
    """The conv Q-net in x3 at the cfg4 act's 8192 rows splits fc1 over K (256 tiles) and its
    learn splits the weight gradients: the K slices are summed in slice order (evx_gemm's
    workspace, splitk_reduce_kernel), so two act calls give the same Q bits, and two learners
    from the same state on the same batch give the same gradients and parameters (ADVICE r2:
    f32 atomics made cfg4's act -- and so its trajectories -- vary between same-seed runs).
    Also against torch fp32 (rtol 2e-4 / atol 2e-5 as test_forward_f32_matches_torch)."""
    _need_gpu()
    from evacx.qnet import Learner
    B = 8192
    g = torch.Generator(device="cuda").manual_seed(8)
    x = (torch.rand(B, 11, 11, 6, device="cuda", generator=g) < 0.3).float()
    x[..., 2] = torch.rand(B, 11, 11, device="cuda", generator=g) * 0.8
    mask = (torch.rand(B, 512, device="cuda", generator=g) >= 0.2).to(torch.uint8)
    lr = Learner(kind="conv", precision="x3", seed=5)
    q1 = lr.q_values(x, train=True, mask=mask).clone()
    q2 = lr.q_values(x, train=True, mask=mask).clone()
    torch.cuda.synchronize()
    assert torch.equal(q1, q2)
    sd = lr.online.state_dict()
    ref = torch_forward("conv", sd, x, mask)
    torch.testing.assert_close(q1, ref, rtol=2e-4, atol=2e-5)
    xb, x2b, a, r, d, m1, m2 = [t.cuda() for t in make_batch(1024, 4)]
    runs = []
    for _ in range(2):
        lrn = Learner(kind="conv", precision="x3", seed=5)
        loss = lrn.learn(xb, a, r, d, x2b, mask_online=m1, mask_target=m2)
        torch.cuda.synchronize()
        runs.append((loss.item(), lrn.grads.flat.clone(), lrn.online.flat.clone()))
    assert runs[0][0] == runs[1][0]
    assert torch.equal(runs[0][1], runs[1][1]) and torch.equal(runs[0][2], runs[1][2])
