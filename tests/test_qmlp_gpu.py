"""GPU numerics of the bf16 MLP fast path (csrc/qmlp.hip) against a plain PyTorch fp32
reference evaluated on the same bf16-rounded operands.

The compact expanded observation (fc1's 484 live inputs: channels 1-4 of every cell;
channel 0 is identically zero, channel 5 the constant centre one-hot folded into the
bias) must equal bf16(evx_obs_expand_f32) exactly on those columns; H1 (bf16
output) may differ from the reference by one bf16 rounding step where the f32
accumulation order changes the rounded value (rtol 1e-2); Q rtol 1e-3 / atol 1e-3.
The actions of the fused epsilon-greedy must equal evx_act on the kernel's own Q."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _env_obs(E=48, steps=7, R=4, grid=48, people=300):
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    lay = DeviceLayout(build_tables(synthetic(grid, grid, R)), people)
    env = VecEnv(lay, E)
    env.seed([77 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(steps):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g))
    torch.cuda.synchronize()
    return lay, env


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("p_drop", [0.0, 0.2])
def test_fused_forward_matches_torch(p_drop):
    _need_gpu()
    from evacx.qmlp import CENTRE_COL, HID, K1, K1P, MLPFast, compact_ref_cols, dropout_keep
    from evacx.qnet import Learner
    lay, env = _env_obs()
    n = env.E * lay.R
    lr = Learner(kind="mlp", precision="bf16", seed=11)
    fast = MLPFast(lr.online, "cuda")
    dev = "cuda"
    h1 = torch.empty(n * HID, dtype=torch.int16, device=dev)
    x = torch.empty(n * K1P, dtype=torch.int16, device=dev)
    h2 = torch.empty(n, 256, device=dev)
    q = torch.empty(n, 5, device=dev)
    act = torch.empty(n, dtype=torch.int32, device=dev)
    drop = (12345, 7, p_drop) if p_drop > 0 else None
    fast.forward(lay.c, env.obs, n, h1, drop=drop, x=x, h2=h2, q=q, actions=act, epsilon=0.3, act_seed=99,
                 act_offset=1000)
    torch.cuda.synchronize()
    # expanded observation: exactly bf16 of the reference tensor
    X = env.expand_obs(torch.float32).reshape(n, K1)
    xk = x.view(torch.bfloat16).view(n, K1P).float()
    cols = torch.from_numpy(compact_ref_cols()).cuda()
    assert torch.equal(xk[:, :cols.numel()], _bf(X)[:, cols])
    assert torch.count_nonzero(xk[:, cols.numel():]) == 0
    # the columns fc1 leaves out: channel 0 all zero, channel 5 the centre one-hot
    assert torch.count_nonzero(X.view(n, 121, 6)[:, :, 0]) == 0
    c5 = torch.zeros(121, device=dev)
    c5[60] = 1.0
    assert torch.equal(X.view(n, 121, 6)[:, :, 5], c5.expand(n, 121))
    assert CENTRE_COL == 60 * 6 + 5
    sd = lr.online.state_dict()
    W1, W2 = _bf(sd["fc1.weight"]), _bf(sd["fc2.weight"])
    ref1 = F.relu(_bf(X) @ W1.t() + sd["fc1.bias"])
    if p_drop > 0:
        keep = torch.from_numpy(dropout_keep(12345, 7, p_drop, n)).to(dev)
        ref1 = torch.where(keep, ref1 / (1 - p_drop), torch.zeros_like(ref1))
        frac = keep.float().mean().item()
        assert abs(frac - (1 - p_drop)) < 0.01, frac
    got1 = h1.view(torch.bfloat16).view(n, HID).float()
    torch.testing.assert_close(got1, _bf(ref1), rtol=1e-2, atol=1e-2)
    # downstream from the kernel's own H1
    ref2 = F.relu(got1 @ W2.t() + sd["fc2.bias"])
    torch.testing.assert_close(h2, ref2, rtol=1e-3, atol=1e-3)
    refq = ref2 @ sd["fc3.weight"].t() + sd["fc3.bias"]
    torch.testing.assert_close(q, refq, rtol=1e-3, atol=1e-3)
    # fused epsilon-greedy == evx_act on the same Q
    from evacx.qnet import qcheck, qlib
    act2 = torch.empty_like(act)
    qcheck(qlib().evx_act(q.data_ptr(), n, 5, 0.3, 99, 1000, act2.data_ptr(), 0), "act")
    torch.cuda.synchronize()
    assert torch.equal(act, act2)


def test_fused_forward_large_batch_runs():
    """Act-sized batch with a ragged tail (N not a multiple of 64)."""
    _need_gpu()
    from evacx.qmlp import HID, MLPFast
    from evacx.qnet import Learner
    lay, env = _env_obs(E=1000, steps=2)
    n = env.E * lay.R - 37
    lr = Learner(kind="mlp", precision="bf16", seed=12)
    fast = MLPFast(lr.online, "cuda")
    h1 = torch.empty(n * HID, dtype=torch.int16, device="cuda")
    q = torch.full((n + 5, 5), 7.0, device="cuda")
    fast.forward(lay.c, env.obs, n, h1, drop=(1, 2, 0.2), q=q)
    torch.cuda.synchronize()
    assert torch.isfinite(q[:n]).all()
    assert torch.all(q[n:] == 7.0)  # nothing written past n


def test_fused_backward_matches_torch_autograd():
    """dW/db of the fused learner vs torch autograd through the same bf16-rounded
    forward (dropout mask = the kernel's hash). The kernels round dZ2/dZ1 to bf16 before
    the weight-gradient GEMMs: max error <= 3e-2 of each gradient's max magnitude."""
    _need_gpu()
    from evacx.qmlp import HID, K1, K1P, MLPFast, dropout_keep
    from evacx.qnet import Learner, qcheck, qlib
    lay, env = _env_obs(E=160, R=4)
    B = 256
    dev = "cuda"
    lr = Learner(kind="mlp", precision="bf16", seed=21)
    fast, fast_t = lr.fast, lr.fast_t
    obs_s = env.obs[:B * 8]
    obs_s2 = env.obs[B * 8:2 * B * 8]
    g = torch.Generator().manual_seed(3)
    a = torch.randint(0, 5, (B,), generator=g, dtype=torch.int32).to(dev)
    r = (torch.randn(B, generator=g) * 10).to(dev)
    done = (torch.rand(B, generator=g) < 0.2).to(torch.uint8).to(dev)
    X = torch.empty(B * K1P, dtype=torch.int16, device=dev)
    H1 = torch.empty(B * HID, dtype=torch.int16, device=dev)
    H2 = torch.empty(B, 256, device=dev)
    Q = torch.empty(B, 5, device=dev)
    H1t = torch.empty(B * HID, dtype=torch.int16, device=dev)
    Qt = torch.empty(B, 5, device=dev)
    dQ = torch.empty(B, 5, device=dev)
    loss = torch.empty(1, device=dev)
    fast.forward(lay.c, obs_s, B, H1, drop=(5, 1, 0.2), x=X, h2=H2, q=Q)
    fast_t.forward(lay.c, obs_s2, B, H1t, drop=(5, 2, 0.2), q=Qt)
    tw = torch.empty(int(qlib().evx_td_loss_ws_floats(B, 1)), device=dev)
    qcheck(qlib().evx_td_loss(Q.data_ptr(), Qt.data_ptr(), 5, a.data_ptr(), r.data_ptr(), done.data_ptr(), 0.99, B,
                              dQ.data_ptr(), loss.data_ptr(), tw.data_ptr(), tw.numel(), 0), "td")
    dz2 = torch.empty(B * 256, dtype=torch.int16, device=dev)
    dz1 = torch.empty(B * HID, dtype=torch.int16, device=dev)
    fast.backward(B, dQ, X, H1, H2, 0.2, dz2, dz1, lr.grads)
    torch.cuda.synchronize()
    # torch reference
    sd = lr.online.state_dict()
    Xf = _bf(env.expand_obs(torch.float32, obs_s).reshape(B, K1))  # the full reference input
    W1 = _bf(sd["fc1.weight"]).requires_grad_()
    b1 = sd["fc1.bias"].clone().requires_grad_()
    W2 = _bf(sd["fc2.weight"]).requires_grad_()
    b2 = sd["fc2.bias"].clone().requires_grad_()
    W3 = sd["fc3.weight"].clone().requires_grad_()
    b3 = sd["fc3.bias"].clone().requires_grad_()
    keep = torch.from_numpy(dropout_keep(5, 1, 0.2, B)).to(dev)
    h1 = torch.where(keep, F.relu(Xf @ W1.t() + b1) / 0.8, torch.zeros(1, device=dev))
    h1 = h1 + (_bf(h1) - h1).detach()  # the kernel stores H1 in bf16
    h2 = F.relu(h1 @ W2.t() + b2)
    q = h2 @ W3.t() + b3
    y = r + 0.99 * Qt.max(1).values * (1 - done.float())
    lref = ((q.gather(1, a.long()[:, None])[:, 0] - y) ** 2).mean()
    lref.backward()
    assert abs(lref.item() - loss.item()) <= 1e-3 * max(1.0, abs(lref.item()))
    for name, ref in [("fc1.weight", W1.grad), ("fc1.bias", b1.grad), ("fc2.weight", W2.grad),
                      ("fc2.bias", b2.grad), ("fc3.weight", W3.grad), ("fc3.bias", b3.grad)]:
        got = lr.grads[name]
        err = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-12)
        assert err < 3e-2, (name, err)
    # every gradient sum goes through partials added in a fixed order: a second run gives
    # every gradient bit for bit
    first = {k: lr.grads[k].clone() for k in lr.grads.shapes}
    fast.backward(B, dQ, X, H1, H2, 0.2, dz2, dz1, lr.grads)
    torch.cuda.synchronize()
    for k, v in first.items():
        assert torch.equal(v, lr.grads[k]), k


def test_learn_obs_step_runs_and_descends():
    """A few fused learn steps on a fixed batch lower the TD loss (Adam lr 1e-3)."""
    _need_gpu()
    from evacx.qnet import Learner
    lay, env = _env_obs(E=160, R=4)
    B = 256
    lr = Learner(kind="mlp", precision="bf16", seed=22, lr=1e-3)
    g = torch.Generator().manual_seed(4)
    a = torch.randint(0, 5, (B,), generator=g, dtype=torch.int32).cuda()
    r = (torch.randn(B, generator=g) * 2).cuda()
    done = torch.ones(B, dtype=torch.uint8).cuda()  # y = r: a fixed regression target
    losses = []
    for _ in range(40):
        losses.append(lr.learn_obs(lay.c, env.obs[:B * 8], a, r, done, env.obs[B * 8:2 * B * 8], B).item())
    assert losses[-1] < 0.5 * losses[0], (losses[0], losses[-1])


@pytest.mark.parametrize("eps", [0.0, 0.25])
def test_fused_act_matches_two_kernel_forward(eps):
    """evx_qmlp_act (H1/H2 on chip, one launch) == evx_qmlp_forward's Q and actions, bit
    for bit, on an act-sized ragged batch with dropout."""
    _need_gpu()
    from evacx.qmlp import HID, MLPFast
    from evacx.qnet import Learner
    lay, env = _env_obs(E=2000, steps=3, R=16, grid=64, people=500)
    n = env.E * lay.R - 7
    lr = Learner(kind="mlp", precision="bf16", seed=31)
    fast = MLPFast(lr.online, "cuda")
    h1 = torch.empty(n * HID, dtype=torch.int16, device="cuda")
    q1 = torch.empty(n, 5, device="cuda")
    a1 = torch.empty(n, dtype=torch.int32, device="cuda")
    q2 = torch.full((n + 3, 5), 9.0, device="cuda")
    a2 = torch.full((n + 3,), -1, dtype=torch.int32, device="cuda")
    kw = dict(drop=(77, 5, 0.2), epsilon=eps, act_seed=4, act_offset=123)
    fast.forward(lay.c, env.obs, n, h1, q=q1, actions=a1, **kw)
    fast.act(lay.c, env.obs, n, q=q2, actions=a2, **kw)
    torch.cuda.synchronize()
    assert torch.equal(q1, q2[:n])
    assert torch.equal(a1, a2[:n])
    assert torch.all(q2[n:] == 9.0) and torch.all(a2[n:] == -1)


def test_static_table_is_fc1_preactivation():
    """evx_qmlp_stat (the act fast path's table) == fc1's pre-activation of the same
    kernel: bf16(relu(T)) equals evx_qmlp_forward's H1 bit for bit on zero-occupancy
    observations at the last fire step (no dropout)."""
    _need_gpu()
    from evacx.qmlp import HID, MLPFast
    from evacx.qnet import Learner
    lay, env = _env_obs(E=8, steps=1, R=4, grid=40, people=100)
    lr = Learner(kind="mlp", precision="bf16", seed=5)
    fast = MLPFast(lr.online, "cuda")
    c = lay.c
    fast.attach_static(c, c.L, c.W, c.t_max)
    ob, T = fast._static[1], fast._static[2]
    n = ob.shape[0]
    assert n == (c.L + 2) * (c.W + 2)
    h1 = torch.empty(n * HID, dtype=torch.int16, device="cuda")
    fast.forward(c, ob, n, h1)
    torch.cuda.synchronize()
    ref = torch.relu(T).to(torch.bfloat16).view(torch.int16).view(-1)
    assert torch.equal(ref, h1)


@pytest.mark.parametrize("eps", [0.0, 0.3])
def test_act_fast_path_matches_full_path(eps):
    """evx_qmlp_act with the static table (tiles whose rows are all at the last fire step
    start fc1 from T[centre] + occupancy columns x bits) vs without it: the same products
    summed in another f32 order, so H1 may differ by one bf16 rounding step -- Q within
    2e-3 of its scale, greedy actions equal on >= 99% of rows. A tile with one row at
    an earlier fire step takes the full path (exact)."""
    _need_gpu()
    from evacx.qmlp import MLPFast
    from evacx.qnet import Learner
    lay, env = _env_obs(E=600, steps=4, R=16, grid=64, people=500)
    c = lay.c
    n = env.E * lay.R - 5
    ob = env.obs.view(-1, 8).clone()
    ob[:, 6] = c.t_max + 3  # past the last fire step (clamped to it)
    ob[130, 6] = 2  # tile 1 (rows 128..255) keeps the full path
    lr = Learner(kind="mlp", precision="bf16", seed=8)
    slow = MLPFast(lr.online, "cuda")
    fastp = MLPFast(lr.online, "cuda")
    fastp.attach_static(c, c.L, c.W, c.t_max)
    kw = dict(drop=(3, 9, 0.2), epsilon=eps, act_seed=11, act_offset=7)
    q1 = torch.empty(n, 5, device="cuda")
    a1 = torch.empty(n, dtype=torch.int32, device="cuda")
    q2 = torch.empty(n, 5, device="cuda")
    a2 = torch.empty(n, dtype=torch.int32, device="cuda")
    slow.act(c, ob, n, q=q1, actions=a1, **kw)
    fastp.act(c, ob, n, q=q2, actions=a2, **kw)
    torch.cuda.synchronize()
    assert torch.equal(q1[128:256], q2[128:256]) and torch.equal(a1[128:256], a2[128:256])
    scale = q1.abs().max().item()
    err = (q1 - q2).abs().max().item()
    assert err <= 2e-3 * scale + 1e-6, (err, scale)
    assert (q1 != q2).any()  # the fast path did run
    agree = (a1 == a2).float().mean().item()
    assert agree >= 0.99, agree
