"""GPU numerics of the f32-accurate (x3) fused MLP kernels (csrc/qmlp.hip) against a plain
PyTorch fp32 reference on the FULL 726-column observation tensor.

x3 carries every f32 operand as bf16 hi + lo (16 significant bits) and a product as
hi*hi + hi*lo + lo*hi with f32 accumulation (~2^-16 relative per product), so the bars
are the exact-f32 path's (tests/test_qnet_gpu.py): Q rtol 2e-4 / atol 2e-5, loss and
gradient norm rtol 2e-4, gradients rtol 2e-3 (atol 1e-5 of the tensor's scale), Adam
updates as test_learn_steps_match_torch_adam. Dropout: explicit keep masks (the same
tensor on both sides) or p = 0."""
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


def torch_q(sd, X, mask):
    """agents/dqn_agent.py:40-61's fc stack on the flattened observation (the MLP variant)."""
    h = F.relu(F.linear(X, sd["fc1.weight"], sd["fc1.bias"]))
    if mask is not None:
        h = h * mask.float() / 0.8
    h = F.relu(F.linear(h, sd["fc2.weight"], sd["fc2.bias"]))
    return F.linear(h, sd["fc3.weight"], sd["fc3.bias"]), h


def _planes(h1, n):
    """f32 value of an x3 activation buffer [2][n][512] (hi + lo)."""
    v = h1.view(torch.bfloat16).view(2, n, -1).float()
    return v[0] + v[1]


@pytest.mark.parametrize("masked", [False, True])
def test_x3_forward_matches_torch_fp32(masked):
    _need_gpu()
    from evacx.qmlp import HID, K1, K1X, MLPFast
    from evacx.qnet import Learner
    lay, env = _env_obs()
    n = env.E * lay.R
    lr = Learner(kind="mlp", precision="f32", seed=11)
    fast = MLPFast(lr.online, "cuda", x3=True)
    dev = "cuda"
    mask = (torch.rand(n, HID, device=dev) >= 0.2).to(torch.uint8) if masked else None
    h1 = torch.empty(2 * n * HID, dtype=torch.int16, device=dev)
    x = torch.empty(n * K1X, dtype=torch.int16, device=dev)
    h2 = torch.empty(n, 256, device=dev)
    q = torch.empty(n, 5, device=dev)
    drop = (1, 2, 0.2, mask) if masked else None
    fast.forward(lay.c, env.obs, n, h1, drop=drop, x=x, h2=h2, q=q)
    torch.cuda.synchronize()
    X = env.expand_obs(torch.float32).reshape(n, K1)
    sd = lr.online.state_dict()
    refq, refh2 = torch_q(sd, X, mask)
    ref1 = F.relu(F.linear(X, sd["fc1.weight"], sd["fc1.bias"]))
    if masked:
        ref1 = ref1 * mask.float() / 0.8
    torch.testing.assert_close(_planes(h1, n), ref1, rtol=2e-4, atol=2e-5)
    torch.testing.assert_close(h2, refh2, rtol=2e-4, atol=2e-5)
    torch.testing.assert_close(q, refq, rtol=2e-4, atol=2e-5)
    # the saved input: the compact features exact, the danger residual slot = the f32 danger's lo
    xv = x.view(torch.bfloat16).view(n, K1X).float()
    from evacx.qmlp import compact_ref_cols
    cols = torch.from_numpy(compact_ref_cols()).to(dev)
    danger = X.view(n, 121, 6)[:, :, 2]
    hi = xv[:, :484].view(n, 121, 4)[:, :, 1]
    assert torch.equal(hi + xv[:, 512:633], hi + (danger - hi).to(torch.bfloat16).float())
    assert ((hi + xv[:, 512:633]) - danger).abs().max().item() <= 2.0 ** -16 * danger.abs().max().item()
    assert torch.equal(xv[:, :484].view(n, 121, 4)[:, :, [0, 2, 3]], X.view(n, 121, 6)[:, :, [1, 3, 4]])
    assert torch.count_nonzero(xv[:, 484:512]) == 0 and torch.count_nonzero(xv[:, 633:]) == 0


@pytest.mark.parametrize("eps", [0.0, 0.25])
def test_x3_act_matches_forward(eps):
    """evx_qmlp_act in x3 mode (qact3: H1 through LDS in two column halves) == the two-kernel
    x3 forward's Q and actions bit for bit (same K order), ragged act-sized batch."""
    _need_gpu()
    from evacx.qmlp import HID, MLPFast
    from evacx.qnet import Learner, qcheck, qlib
    lay, env = _env_obs(E=700, steps=3, R=16, grid=64, people=500)
    n = env.E * lay.R - 7
    lr = Learner(kind="mlp", precision="f32", seed=31)
    fast = lr.fast
    assert fast.x3
    h1 = torch.empty(2 * n * HID, dtype=torch.int16, device="cuda")
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
    a3 = torch.empty_like(a1)
    qcheck(qlib().evx_act(q1.data_ptr(), n, 5, eps, 4, 123, a3.data_ptr(), 0), "act")
    torch.cuda.synchronize()
    assert torch.equal(a1, a3)


def test_x3_learn_steps_match_torch_adam():
    """3 fused learn steps (learn_obs, x3): loss, gradient norm, clipped gradients, Adam
    parameters vs torch autograd in fp32 on the expanded observations, same masks."""
    _need_gpu()
    from evacx.qmlp import HID, K1
    from evacx.qnet import Learner
    lay, env = _env_obs(E=160, R=4)
    B = 256
    dev = "cuda"
    lr = Learner(kind="mlp", precision="f32", seed=21, lr=1e-3)
    sd0 = {k: v.clone() for k, v in lr.online.state_dict().items()}
    params = {k: torch.nn.Parameter(v.clone()) for k, v in sd0.items()}
    tgt = {k: v.clone() for k, v in sd0.items()}
    opt = torch.optim.Adam(params.values(), lr=1e-3)
    g = torch.Generator().manual_seed(3)
    for it in range(3):
        if it > 0:  # each step compared from the same state (params + moments)
            lr.online.load_state_dict({k: p.detach() for k, p in params.items()})
            lr.fast.repack()
            for key, buf in (("exp_avg", lr.m), ("exp_avg_sq", lr.v)):
                buf.copy_(torch.cat([opt.state[p][key].reshape(-1) for p in params.values()]))
        perm = torch.randperm(env.E * lay.R, generator=g)
        s_idx, s2_idx = perm[:B].to(dev), perm[B:2 * B].to(dev)
        obs = env.obs.view(-1, 8)
        s_obs, s2_obs = obs[s_idx].contiguous().view(-1), obs[s2_idx].contiguous().view(-1)
        a = torch.randint(0, 5, (B,), generator=g, dtype=torch.int32).to(dev)
        r = (torch.randn(B, generator=g) * 30).to(dev)
        d = (torch.rand(B, generator=g) < 0.2).to(torch.uint8).to(dev)
        m1 = (torch.rand(B, HID, generator=g) >= 0.2).to(torch.uint8).to(dev)
        m2 = (torch.rand(B, HID, generator=g) >= 0.2).to(torch.uint8).to(dev)
        loss = lr.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B, mask_online=m1, mask_target=m2)
        X = env.expand_obs(torch.float32, s_obs).reshape(B, K1)
        X2 = env.expand_obs(torch.float32, s2_obs).reshape(B, K1)
        q = torch_q(params, X, m1)[0].gather(1, a.long().unsqueeze(1))
        with torch.no_grad():
            y = r + 0.99 * torch_q(tgt, X2, m2)[0].max(1)[0] * (~d.bool())
        ref_loss = F.mse_loss(q.squeeze(), y)
        opt.zero_grad()
        ref_loss.backward()
        gnorm = torch.nn.utils.clip_grad_norm_(params.values(), 1.0)
        grads_ref = {k: p.grad.clone() for k, p in params.items()}
        opt.step()
        torch.cuda.synchronize()
        assert abs(loss.item() - ref_loss.item()) <= 2e-4 * abs(ref_loss.item()) + 1e-5
        assert abs(lr.norm.item() - gnorm.item()) <= 2e-4 * gnorm.item() + 1e-6
        for k in params:
            ref = grads_ref[k]
            torch.testing.assert_close(lr.grads[k], ref, rtol=2e-3, atol=1e-5 * ref.abs().max().item() + 1e-9)
            diff = (lr.online[k] - params[k].detach()).abs()
            assert (diff > 1e-5).float().mean().item() <= 1e-3, (k, diff.max().item())
            assert diff.max().item() <= 2e-3, (k, diff.max().item())


def test_x3_layout_set_reads_each_rows_layout():
    """x3 forward over a LayoutSet: every row's danger residual comes from its own layout."""
    _need_gpu()
    from evacx.env import DeviceLayout, LayoutSet, VecEnv
    from evacx.layout import build_tables, random_layout
    from evacx.qmlp import HID, K1
    from evacx.qnet import Learner
    E, R, P = 30, 4, 200
    lays = LayoutSet([DeviceLayout(build_tables(random_layout(40, 40, R, 900 + k)), P) for k in range(3)])
    env = VecEnv(lays, E, layout_of=[e % 3 for e in range(E)])
    env.seed([5 + i for i in range(E)])
    env.reset()
    for _ in range(4):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32))
    n = E * R
    lr = Learner(kind="mlp", precision="f32", seed=2)
    h1 = torch.empty(2 * n * HID, dtype=torch.int16, device="cuda")
    q = torch.empty(n, 5, device="cuda")
    lr.fast.forward(lays.c, env.obs, n, h1, q=q)
    torch.cuda.synchronize()
    X = env.expand_obs(torch.float32).reshape(n, K1)
    refq, _ = torch_q(lr.online.state_dict(), X, None)
    torch.testing.assert_close(q, refq, rtol=2e-4, atol=2e-5)


def test_x3_rejects_missing_operands():
    """The product path fails loudly when the x3 operands are absent."""
    _need_gpu()
    from evacx import _lib
    from evacx.qmlp import HID, MLPFast
    from evacx.qnet import Learner
    lay, env = _env_obs(E=4, steps=1)
    lr = Learner(kind="mlp", precision="f32", seed=1)
    fast = MLPFast(lr.online, "cuda", x3=True)
    fast.c.w1l = None
    with pytest.raises(_lib.EvacxError):
        fast.forward(lay.c, env.obs, 16, torch.empty(2 * 16 * HID, dtype=torch.int16, device="cuda"),
                     q=torch.empty(16, 5, device="cuda"))


@pytest.mark.parametrize("hook", [False, True])
def test_fused_learn_chain_matches_separate_launches(hook):
    """The collapsed x3 learn chain (TD + gradient clear in one launch; qdz1 + dW2 in one launch;
    both split-K reductions + clip_grad_norm_'s squared-norm partials in one launch; clip + Adam
    + operand repack in one launch, evx_qmlp_adam_pack3) against the separate launches (td_loss,
    zero, qdz1, gemm_tn + reduce x2, sumsq, clip_adam, pack3) from the same state over three
    learn steps: loss, norm, clipped gradients and parameters within f32 reassociation; the
    fused kernel's bf16 hi / lo operand tiles and b1c bit-identical to pack3 of its own updated
    parameters. hook: a gradient hook (the multi-GPU all-reduce's slot) makes the norm partials
    come from a pass over the flat gradients instead (evx_qmlp_sumsq_parts)."""
    _need_gpu()
    from evacx.qmlp import HID
    from evacx.qnet import Learner
    lay, env = _env_obs(E=320, R=4)
    B = 512
    assert 2 * B <= env.E * lay.R
    dev = "cuda"
    runs = []
    for fused in (False, True, True):
        lr = Learner(kind="mlp", precision="f32", seed=33, lr=1e-3)
        lr.fused_opt = fused
        if hook:
            lr.grad_hook = lambda g: g.mul_(1.0)
        g = torch.Generator().manual_seed(9)
        for it in range(3):
            perm = torch.randperm(env.E * lay.R, generator=g)
            obs = env.obs.view(-1, 8)
            s_obs = obs[perm[:B].to(dev)].contiguous().view(-1)
            s2_obs = obs[perm[B:2 * B].to(dev)].contiguous().view(-1)
            a = torch.randint(0, 5, (B,), generator=g, dtype=torch.int32).to(dev)
            r = (torch.randn(B, generator=g) * 30).to(dev)
            d = (torch.rand(B, generator=g) < 0.2).to(torch.uint8).to(dev)
            m1 = (torch.rand(B, HID, generator=g) >= 0.2).to(torch.uint8).to(dev)
            m2 = (torch.rand(B, HID, generator=g) >= 0.2).to(torch.uint8).to(dev)
            loss = lr.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B, mask_online=m1, mask_target=m2)
        torch.cuda.synchronize()
        runs.append(dict(loss=loss.item(), norm=lr.norm.item(),
                         grads={k: v.clone() for k, v in lr.grads.state_dict().items()},
                         params={k: v.clone() for k, v in lr.online.state_dict().items()},
                         packed=[t.clone() for t in (lr.fast.w1b, lr.fast.w1l, lr.fast.b1c, lr.fast.w2b, lr.fast.w2l,
                                                     lr.fast.w2t, lr.fast.w2tl)], lr=lr))
    sep, fus, fus2 = runs
    # the same seed and batches give the same bits (every gradient sum in a fixed order)
    assert fus["loss"] == fus2["loss"] and fus["norm"] == fus2["norm"]
    for k in fus["params"]:
        assert torch.equal(fus["grads"][k], fus2["grads"][k]), k
        assert torch.equal(fus["params"][k], fus2["params"][k]), k
    assert abs(sep["loss"] - fus["loss"]) <= 1e-5 * abs(sep["loss"]) + 1e-7
    assert abs(sep["norm"] - fus["norm"]) <= 1e-5 * sep["norm"] + 1e-9
    for k in sep["params"]:
        scale = sep["grads"][k].abs().max().item()
        # after three Adam steps the two chains differ only by the reassociation of the gradient
        # norm's f32 sum (norm partials of reduce2 vs sumsq_parts)
        torch.testing.assert_close(fus["grads"][k], sep["grads"][k], rtol=1e-4, atol=1e-6 * scale + 1e-12)
        torch.testing.assert_close(fus["params"][k], sep["params"][k], rtol=1e-5, atol=2e-6)
    lr = fus["lr"]
    lr.fast.repack()  # pack3 of the fused run's own parameters
    torch.cuda.synchronize()
    for got, want in zip(fus["packed"], (lr.fast.w1b, lr.fast.w1l, lr.fast.b1c, lr.fast.w2b, lr.fast.w2l,
                                         lr.fast.w2t, lr.fast.w2tl)):
        assert torch.equal(got, want)


@pytest.mark.parametrize("grid,xr", [(48, "all"), (128, "robot_range")])
def test_x3_static_table_vs_float64(grid, xr):
    """evx_qmlp_stat in x3 (the act table: fc1's pre-activation, bias included) against the same in
    float64 on the table's own observations (every window centre at the last fire step, zero
    occupancy), within the x3 products' 2^-16 relative rounding: grid 48 over every centre (a
    ragged last row tile), grid 128 over Map.robot_range's columns (the trainer's table)."""
    _need_gpu()
    from evacx.qmlp import K1
    from evacx.qnet import Learner
    lay, env = _env_obs(E=8, steps=2, R=2, grid=grid, people=300)
    c = lay.c
    lr = Learner(kind="mlp", precision="f32", seed=41)
    x_range = (max(int(c.rx_lo), 0), min(int(c.rx_hi), int(c.L) + 1)) if xr == "robot_range" else None
    lr.fast.attach_static(c, int(c.L), int(c.W), int(c.t_max), x_range=x_range)
    ob, T = lr.fast._static[1], lr.fast._static[2]
    n = ob.shape[0]
    # the rebuild reads the rows' X expanded once (evx_qmlp_stat_x): the table generated from the
    # observations (evx_qmlp_stat) is the same bit for bit
    assert lr.fast._static_x is not None
    T_gen = torch.empty_like(T)
    lr.fast.stat_table(c, ob, n, T_gen)
    torch.cuda.synchronize()
    assert torch.equal(T, T_gen)
    X = env.expand_obs(torch.float32, ob.reshape(-1)).reshape(n, K1).double()
    sd = lr.online.state_dict()
    W1, b1 = sd["fc1.weight"].double(), sd["fc1.bias"].double()
    ref = X @ W1.t() + b1
    bound = X.abs() @ W1.abs().t() + b1.abs()  # |terms|: the x3 rounding is relative to them
    err = (T.double() - ref).abs()
    assert torch.isfinite(T).all()
    assert (err <= 4e-5 * bound + 1e-7).all(), float((err / (bound + 1e-12)).max())


@pytest.mark.parametrize("xr", ["all", "robot_range"])
def test_x3_act_static_table_and_env_order(xr):
    """x3 act fast path: rows whose fire has reached the layout's last step start fc1 from the
    per-centre table of the static features (evx_qmlp_stat, x3) and add the occupancy columns
    (hi + lo weights); VecEnv.act_perm visits those envs first so act tiles are uniform.
    Against the plain x3 act on the same observations: Q within f32 reassociation (and not
    bit-identical on the table rows: the table path ran), greedy actions equal, epsilon draws
    and dropout rows keyed by the original row (epsilon = 1: identical actions); act_perm is
    the stable partition of the envs by fire step >= t_max. robot_range: the table covers only
    the centres of Map.robot_range's columns (the trainer's table)."""
    _need_gpu()
    from evacx.qnet import DROPOUT_P, Learner
    lay, env = _env_obs(E=256, R=4)
    E, R, n = 256, 4, 256 * 4
    t_max = int(lay.c.t_max)
    sat = torch.tensor([e % 3 != 0 for e in range(E)], device="cuda")
    # envs past the fire's last step: their scalar fire step and their observations' fire step
    env.scal.view(E, 4)[:, 0] = torch.where(sat, torch.full_like(env.scal.view(E, 4)[:, 0], t_max),
                                            env.scal.view(E, 4)[:, 0])
    ob = env.obs.view(E, R, 8)
    ob[:, :, 6] = torch.where(sat[:, None], torch.full_like(ob[:, :, 6], t_max), ob[:, :, 6])
    env.refresh_classes()  # the class bytes act_perm reads follow the state words written here
    perm = torch.full((E,), -1, dtype=torch.int32, device="cuda")
    env.act_perm(perm)
    torch.cuda.synchronize()
    s = sat.cpu().numpy()
    want = np.concatenate([np.nonzero(s)[0], np.nonzero(~s)[0]])
    assert np.array_equal(perm.cpu().numpy(), want)
    lr = Learner(kind="mlp", precision="f32", seed=3)
    fast = lr.fast
    obs = env.obs.view(-1)
    res = {}
    for mode in ("plain", "table"):
        if mode == "table":
            x_range = (int(lay.c.rx_lo), int(lay.c.rx_hi)) if xr == "robot_range" else None
            fast.attach_static(lay.c, int(lay.c.L), int(lay.c.W), t_max, x_range=x_range)
            if x_range is not None:
                assert fast._static[2].shape[0] == (x_range[1] - x_range[0] + 1) * (int(lay.c.W) + 2)
        kw = dict(perm=perm, rows_per_env=R) if mode == "table" else {}
        q = torch.empty(n, 5, device="cuda")
        a0 = torch.empty(n, dtype=torch.int32, device="cuda")
        a1 = torch.empty(n, dtype=torch.int32, device="cuda")
        fast.act(lay.c, obs, n, drop=(9, 4, DROPOUT_P), q=q, actions=a0, epsilon=0.0, **kw)
        fast.act(lay.c, obs, n, drop=(9, 4, DROPOUT_P), actions=a1, epsilon=1.0, act_seed=5, act_offset=77, **kw)
        torch.cuda.synchronize()
        res[mode] = (q, a0, a1)
    (qp, ap0, ap1), (qt, at0, at1) = res["plain"], res["table"]
    scale = qp.abs().max().item()
    assert (qt - qp).abs().max().item() <= 2e-5 * scale
    rows_sat = sat.repeat_interleave(R)
    assert not torch.equal(qt[rows_sat], qp[rows_sat])  # the table path ran on those rows
    assert torch.equal(qt[~rows_sat], qp[~rows_sat])    # the full path, same rows: bit for bit
    assert (at0 == ap0).float().mean().item() >= 0.99
    assert torch.equal(at1, ap1)


def test_x3_act_at_bench_rows_table_path_env_order():
    """The act as the cfg3 bench runs it: 524 288 rows (32 768 envs x 16 robots), the per-centre
    table path for the envs past the fire's last step (85 %), VecEnv.act_perm's env order, dropout
    and epsilon = 0.1 (agents/dqn_agent.py:101-124). Real 128x128 R16 observations (4096 envs, a few
    steps) tiled 8 times, fire step raised to t_max on 85 % of the envs. Q of a sample of 64 runs of
    64 rows against torch fp32 on the expanded observations with the kernel's own dropout masks
    (rtol 2e-4, atol 1e-4 of the Q scale: the x3 bars plus the table path's reassociation);
    actions = the epsilon-greedy restatement (oracle.epsilon_greedy) of the kernel's Q on every row,
    and the greedy argmax of torch's Q on >= 99.5 % of the sampled rows."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qmlp import HID, K1, dropout_keep
    from evacx.qnet import DROPOUT_P, Learner
    from oracle import oracle as orc
    R, E0, rep = 16, 4096, 8
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), 2276)
    env = VecEnv(lay, E0)
    env.seed([900 + i for i in range(E0)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(4):
        env.step(torch.randint(0, 5, (E0 * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    torch.cuda.synchronize()
    E, n = E0 * rep, E0 * rep * R
    t_max = int(lay.c.t_max)
    obs = env.obs.view(E0, R, 8).repeat(rep, 1, 1).contiguous()
    rng = np.random.RandomState(5)
    sat = torch.from_numpy(rng.rand(E) < 0.85).cuda()
    obs[:, :, 6] = torch.where(sat[:, None], torch.full_like(obs[:, :, 6], t_max), obs[:, :, 6])
    s = sat.cpu().numpy()
    perm = torch.from_numpy(np.concatenate([np.nonzero(s)[0], np.nonzero(~s)[0]]).astype(np.int32)).cuda()
    lr = Learner(kind="mlp", precision="f32", seed=41)
    fast = lr.fast
    lc = lay.c
    fast.attach_static(lc, int(lc.L), int(lc.W), t_max, x_range=(max(lc.rx_lo, 0), min(lc.rx_hi, lc.L + 1)))
    q = torch.empty(n, 5, device="cuda")
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    seed, stream, eps, aseed, aoff = 12, 7, 0.1, 4, 1000
    fast.act(lc, obs.view(-1), n, drop=(seed, stream, DROPOUT_P), q=q, actions=a, epsilon=eps, act_seed=aseed,
             act_offset=aoff, perm=perm, rows_per_env=R)
    torch.cuda.synchronize()
    qk = q.cpu().numpy()
    assert np.array_equal(a.cpu().numpy(), orc.epsilon_greedy(qk, eps, aseed, aoff))
    starts = np.sort(rng.choice(n // 64, 64, replace=False)) * 64
    rows = np.concatenate([np.arange(r0, r0 + 64) for r0 in starts])
    ob_s = obs.view(n, 8)[torch.from_numpy(rows).cuda()].contiguous()
    X = env.expand_obs(torch.float32, ob_s.view(-1)).reshape(len(rows), K1)
    keep = np.concatenate([dropout_keep(seed, stream, DROPOUT_P, 64, HID, row0=int(r0)) for r0 in starts])
    mask = torch.from_numpy(keep.astype(np.uint8)).cuda()
    refq, _ = torch_q(lr.online.state_dict(), X, mask)
    got = q[torch.from_numpy(rows).cuda()]
    scale = refq.abs().max().item()
    torch.testing.assert_close(got, refq, rtol=2e-4, atol=1e-4 * scale)
    assert (got.argmax(1) == refq.argmax(1)).float().mean().item() >= 0.995
    # the table path ran on the saturated envs' rows (not bit-identical to the full path there)
    assert s[rows // R].any()


@pytest.mark.parametrize("case", ["bench_rows_perm", "ragged_no_dropout", "all_full_path"])
def test_x3_persistent_act_matches_64_row_kernel(case):
    """evx_qmlp_act's persistent 128-row kernel (qact3p_kernel: one workgroup per CU, fc1 quarters
    pipelined against fc2, H1^T in swizzled LDS read by ds_read_b64_tr_b16) against the 64-row kernel
    (evx_qmlp_act64) on the same inputs: Q and epsilon-greedy actions bit for bit.
    bench_rows_perm: 524 288 rows (32 768 envs x 16 robots), 85 % of the envs at the table's fire step
    first in the act order (the boundary tiles and the rest take the fallback, act3h_tile), hash
    dropout, epsilon 0.1; ragged_no_dropout: 2048 x 128 + 72 rows, every row on the table path, no
    perm, p = 0 (the DM 0 instantiation, a partial last tile); all_full_path: 262 144 rows with no row at
    the table's fire step (every tile through the fallback)."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qnet import DROPOUT_P, Learner
    R, E0 = 16, 2048
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), 2276)
    env = VecEnv(lay, E0)
    env.seed([300 + i for i in range(E0)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(8)
    for _ in range(6):
        env.step(torch.randint(0, 5, (E0 * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    torch.cuda.synchronize()
    t_max = int(lay.c.t_max)
    lr = Learner(kind="mlp", precision="f32", seed=17)
    fast, lc = lr.fast, lay.c
    fast.attach_static(lc, int(lc.L), int(lc.W), t_max, x_range=(max(lc.rx_lo, 0), min(lc.rx_hi, lc.L + 1)))
    kw, drop, eps = {}, (21, 5, DROPOUT_P), 0.1
    if case == "bench_rows_perm":
        rep = 16
        E, n = E0 * rep, E0 * rep * R
        obs = env.obs.view(E0, R, 8).repeat(rep, 1, 1).contiguous()
        sat = torch.from_numpy(np.random.RandomState(2).rand(E) < 0.85).cuda()
        obs[:, :, 6] = torch.where(sat[:, None], torch.full_like(obs[:, :, 6], t_max), obs[:, :, 6])
        s = sat.cpu().numpy()
        perm = torch.from_numpy(np.concatenate([np.nonzero(s)[0], np.nonzero(~s)[0]]).astype(np.int32)).cuda()
        kw = dict(perm=perm, rows_per_env=R)
    elif case == "ragged_no_dropout":
        n = 8 * 256 * 128 + 72  # >= 4 tiles per CU (the persistent kernel's threshold)
        obs = env.obs.view(-1, 8).repeat(9, 1)[:n].contiguous()
        obs[:, 6] = t_max
        drop = (21, 5, 0.0)
    else:
        rep = 8
        n = E0 * rep * R
        obs = env.obs.view(-1, 8).repeat(rep, 1).contiguous()
        obs[:, 6] = torch.clamp(obs[:, 6], max=t_max - 1)
    from evacx.qmlp import act_ws_ints
    ws = torch.zeros(act_ws_ints(n), dtype=torch.int32, device="cuda")
    out = {}
    # the persistent kernel without a workspace (its fallback re-checks every row), with one (the
    # tiles off the table path listed; twice on the same workspace, whose counters each act resets),
    # and the 64-row kernel
    for key, k64, w in (("p", False, None), ("pw", False, ws), ("pw2", False, ws), ("k64", True, None)):
        q = torch.full((n, 5), float("nan"), device="cuda")
        a = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        fast.act(lc, obs.view(-1), n, drop=drop, q=q, actions=a, epsilon=eps, act_seed=6, act_offset=33,
                 kernel64=k64, ws=w, **kw)
        torch.cuda.synchronize()
        out[key] = (q, a)
        if w is not None:
            assert w[:2].tolist() == [0, 0]  # the count and the done counter, reset for the next act
    q6, a6 = out["k64"]
    assert torch.isfinite(q6).all() and (a6 >= 0).all()
    for key in ("p", "pw", "pw2"):
        qp, ap = out[key]
        assert torch.equal(qp, q6), key
        assert torch.equal(ap, a6), key
