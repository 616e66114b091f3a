"""Parity of the kernels at the sizes bench.py times them (VERDICT r2 "Next round" 1).

The kernel variant a launch picks depends on its size, so parity at small E / small B
says nothing about the variant the bench runs:

* env.step: evx_env_step picks one-wave workgroups at E >= 64 x CUs (32 x CUs for big grids;
  env_step_kernel<1, ...>, csrc/env_step.hip: evx_env_step_part), 4-wave workgroups with the
  heavy-env path below: cfg4's 256x256 grid at 8192 envs runs the big-grid instantiation
  <1, false, true>, cfg5's 8192 envs the 4-wave path (cfg3's 32768-env one-wave launch:
  tests/test_env_gpu.py::test_env_parity_bench_scale). cfg4 (256x256, P 9102, R 1, 8192 envs)
  and cfg5 (128x128, P 2276, R 32, 8192 envs) are prepared as bench.py prepares them
  (env-only steps, env g force-reset at step g % stagger: ages spread over an episode,
  fused auto-resets), then envs spread over the age mix are snapshotted into the oracle
  (oracle/evac_oracle.c, pinned by the reference's trajectories) and both step with the
  same actions: every state field, both MT19937 streams, reward, done and observation
  (terminal ones through obs_term) bit-exact on every step.
  Reference: envs/people.py:196-314, envs/evacuation_env.py:84-288.

* learn: the x3 learn chain at the bench's batches: the online forward alone through
  qfc1_kernel<2,2,4,true> (64 x 256 tiles) + qfc23, the target through the fused act kernel
  at B >= 32768 (qact3h_kernel), multi-tile qdz1 workgroups (8 tiles at B = 32768, 2 at 8192;
  csrc/qmlp.hip: qdz1_tiles_per_wg, launch_fwd, evx_qmlp_forward2). One DQNAgent.learn step
  (agents/dqn_agent.py:126-168) from compact observations of a 128x128 R16 env, explicit
  dropout keep masks, against torch fp32 autograd + clip_grad_norm_ + Adam on the expanded
  observations -- the same restatement tests/test_dqn_golden_cpu.py pins to the reference's
  own dqn_learn.npz. Tolerances are the x3 path's (tests/test_qmlp_x3_gpu.py): loss and
  norm rtol 2e-4, gradients rtol 2e-3 with atol 1e-5 of the tensor's max, Adam parameters
  within 2e-3 of lr-scale and at most 0.1 % beyond 1e-5.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _prepare_like_bench(env, E, R, age_steps, stagger, seed=4321):
    """bench.py's --phase stationary preparation (uniform random actions, staggered resets)."""
    gid = torch.arange(E, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(seed)
    acts = torch.empty(E * R, device="cuda", dtype=torch.int32)
    for w in range(age_steps):
        torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g, out=acts)
        env.step(acts, auto_reset=True)
        if w < stagger:
            env.reset(mask=(gid % stagger == w) & ~env.done.bool())


def _bench_mix_parity(L, P, R, E, age_steps, stagger, n_snap, steps, min_age_span):
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from oracle import oracle as orc
    tables = build_tables(synthetic(L, L, R))
    lay = DeviceLayout(tables, P)
    env = VecEnv(lay, E)
    env.seed([1234 + i for i in range(E)])
    env.reset()
    _prepare_like_bench(env, E, R, age_steps, stagger)
    ids = list(range(0, E, E // n_snap))[:n_snap]
    olay = orc.Layout.from_tables(tables, P)
    oenvs = []
    for st in env.host_states(ids):
        oe = orc.Env(olay, thmap=False)
        oe.load_state(st)
        oenvs.append(oe)
    ages = np.array([oe.scal[1] for oe in oenvs])
    assert ages.max() - ages.min() >= min_age_span, ages  # the sample spans the episode-age mix
    rng = np.random.RandomState(11)
    n_done = 0
    idt = torch.tensor(ids, device="cuda")
    for s in range(steps):
        a = rng.randint(0, 5, size=(E, R)).astype(np.int32)
        a[rng.rand(E, R) < 0.02] = 7  # invalid actions: silent no-ops (envs/map.py:180-181)
        env.step(torch.from_numpy(a.reshape(-1)).cuda(), auto_reset=True)
        rew = env.reward[ids].cpu().numpy()
        dn = env.done[ids].cpu().numpy()
        ob = env.expand_obs(torch.float64, env.obs.view(E, -1)[idt].reshape(-1)).cpu().numpy()
        term = env.expand_obs(torch.float64, env.obs_term.view(E, -1)[idt].reshape(-1)).cpu().numpy() \
            if dn.any() else None
        sts = env.host_states(ids)
        for j, (e, oe) in enumerate(zip(ids, oenvs)):
            oobs, r, d = oe.step(a[e])
            assert rew[j] == r and bool(dn[j]) == d, (s, e, rew[j], r)
            if d:
                assert np.array_equal(term[j], oobs), (s, e, "terminal obs")
                oobs = oe.reset()
                n_done += 1
            assert np.array_equal(ob[j], oobs), (s, e, "obs")
            st = sts[j]
            for k in ["pos", "flags", "health", "acc", "rmap", "robots", "view", "scal", "py_mt", "np_mt"]:
                assert np.array_equal(st[k], getattr(oe, k)), (s, e, k)
    env.check_err()
    return ages, n_done


def test_cfg4_env_at_bench_scale():
    """cfg4: 256x256, P 9102, R 1, 8192 envs (env_step_kernel<1, false, true>), prepared as the
    cfg4 bench line (--age-steps 300 --stagger 300); 32 envs x 40 steps vs the oracle."""
    _need_gpu()
    ages, _ = _bench_mix_parity(L=256, P=9102, R=1, E=8192, age_steps=300, stagger=300, n_snap=32, steps=40,
                                min_age_span=200)
    print(f"cfg4 bench mix: ages {ages.min()}..{ages.max()}")


def test_cfg5_env_at_bench_scale():
    """cfg5: 128x128, P 2276, R 32, 8192 envs (4-wave workgroups, heavy-env path), prepared as the bench
    (--age-steps 1300 --stagger 1200); 48 envs x 50 steps vs the oracle."""
    _need_gpu()
    ages, n_done = _bench_mix_parity(L=128, P=2276, R=32, E=8192, age_steps=1300, stagger=1200, n_snap=48,
                                     steps=50, min_age_span=600)
    print(f"cfg5 bench mix: ages {ages.min()}..{ages.max()}, resets {n_done}")


# ------------------------------------------------------------------------- learn
def _torch_q(sd, X, mask):
    h = F.relu(F.linear(X, sd["fc1.weight"], sd["fc1.bias"]))
    if mask is not None:
        h = h * mask.float() / 0.8
    h = F.relu(F.linear(h, sd["fc2.weight"], sd["fc2.bias"]))
    return F.linear(h, sd["fc3.weight"], sd["fc3.bias"])


def _torch_q_gated(sd, X, g1, g2):
    """The same network with the ReLU/dropout pattern given (g1: keep AND fc1 > 0, g2: fc2 > 0) --
    the device's own pattern, so autograd walks the branches the device's backward walked."""
    z1 = F.linear(X, sd["fc1.weight"], sd["fc1.bias"])
    h1 = z1 * g1 / 0.8
    z2 = F.linear(h1, sd["fc2.weight"], sd["fc2.bias"])
    return F.linear(z2 * g2, sd["fc3.weight"], sd["fc3.bias"]), z1, z2


@pytest.mark.parametrize("B,table", [(8192, False), (8192, True), (32768, False), (32768, True)])
def test_x3_learn_at_bench_batch(B, table):
    """Two learn steps (each from the same parameters and Adam moments on both sides) at the
    bench's learn batch: cfg5's 8192 (2-tile qdz1) and cfg3's 32768 (8-tile qdz1); the online
    forward through qfc1<2,2,4,true> + qfc23, or (table: as VecTrainer runs it, the online net
    with its act table) through x_expand_kernel + qact3h_kernel SAVE (B = 8192: both nets in one
    qfwd2_kernel launch), with three quarters of the s and s' rows moved to the layout's last fire
    step so their tiles start fc1 from the tables.
    Observations: a 128x128 R16 env 40 steps into its episode (fire spreading, people moving),
    sampled without replacement into s and s'.

    ReLU branches. x3 products are ~2^-17 off, so a pre-activation within that of 0 can take
    the other ReLU branch than fp32 torch; at these batches (16.8 M fc1 and 8.4 M fc2
    activations at B = 32768) a few do, and each moves its row's whole contribution to the
    gradients (tools/learn_diag.py: up to 1e-2 of max |grad| in db1 and the occupancy columns).
    So (1) every activation whose branch differs from torch's must have a torch pre-activation
    within 1e-4 of the layer's max |z| (the x3 rounding of 0), and at most 1e-5 of them may
    differ; (2) the gradients, norm and Adam update are compared with the tests' x3 tolerances
    against torch autograd through the DEVICE's branch pattern (read from the saved H1 / H2), so
    the arithmetic is checked to 2e-3 / 1e-5 of max |grad|; (3) against plain torch the loss
    (rtol 2e-4) and the norm (rtol 1e-3)."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qmlp import HID, HID2, K1
    from evacx.qnet import Learner
    R, P = 16, 2276
    E = 2 * B // R
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), P)
    env = VecEnv(lay, E)
    env.seed([500 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(40):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    torch.cuda.synchronize()
    dev = "cuda"
    lr = Learner(kind="mlp", precision="f32", seed=41, lr=1e-3)
    assert lr.fast is not None and lr.fast.x3 and lr.fused_opt  # the trainer's chain
    c = lay.c
    if table:  # both nets' act tables, as VecTrainer attaches them
        lr.fast.attach_static(c, c.L, c.W, c.t_max, x_range=(max(c.rx_lo, 0), min(c.rx_hi, c.L + 1)))
        lr.fast_t.attach_static(c, c.L, c.W, c.t_max, x_range=(max(c.rx_lo, 0), min(c.rx_hi, c.L + 1)))
    sd0 = {k: v.clone() for k, v in lr.online.state_dict().items()}
    params = {k: torch.nn.Parameter(v.clone()) for k, v in sd0.items()}
    tgt = {k: v.clone() for k, v in sd0.items()}
    opt = torch.optim.Adam(params.values(), lr=1e-3)
    gh = torch.Generator().manual_seed(B)
    obs = env.obs.view(-1, 8)
    n_flips = 0
    for it in range(2):
        if it > 0:
            lr.online.load_state_dict({k: p.detach() for k, p in params.items()})
            lr.fast.repack()
            for key, buf in (("exp_avg", lr.m), ("exp_avg_sq", lr.v)):
                buf.copy_(torch.cat([opt.state[p][key].reshape(-1) for p in params.values()]))
        perm = torch.randperm(E * R, generator=gh)
        s_obs = obs[perm[:B].to(dev)].contiguous()
        if table:
            s_obs[:3 * B // 4, 6] = int(c.t_max)
        s_obs = s_obs.view(-1)
        s2_obs = obs[perm[B:2 * B].to(dev)].contiguous()
        if table:
            s2_obs[B // 4:, 6] = int(c.t_max)
        s2_obs = s2_obs.view(-1)
        a = torch.randint(0, 5, (B,), generator=gh, dtype=torch.int32).to(dev)
        r = (torch.randn(B, generator=gh) * 30).to(dev)
        d = (torch.rand(B, generator=gh) < 0.05).to(torch.uint8).to(dev)
        m1 = (torch.rand(B, HID, generator=gh) >= 0.2).to(torch.uint8).to(dev)
        m2 = (torch.rand(B, HID, generator=gh) >= 0.2).to(torch.uint8).to(dev)
        loss = lr.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B, mask_online=m1, mask_target=m2)
        torch.cuda.synchronize()
        # the device's branch pattern, from the forward it saved for the backward
        h1 = lr.net.ws.get("fh1", (2 * B * HID,), torch.int16, torch.device(dev)).view(torch.bfloat16)
        h1 = h1.view(2, B, HID).float().sum(0)
        h2 = lr.net.ws.get("fh2", (B * HID2,), torch.float32, torch.device(dev)).view(B, HID2)
        g1, g2 = (h1 > 0).float(), (h2 > 0).float()
        X = env.expand_obs(torch.float32, s_obs).reshape(B, K1)
        X2 = env.expand_obs(torch.float32, s2_obs).reshape(B, K1)
        with torch.no_grad():
            y = r + 0.99 * _torch_q(tgt, X2, m2).max(1)[0] * (~d.bool())
            # (3) plain torch: loss and norm
            plain = {k: p.detach().clone().requires_grad_(True) for k, p in params.items()}
        q_plain = _torch_q(plain, X, m1).gather(1, a.long().unsqueeze(1))
        F.mse_loss(q_plain.squeeze(), y).backward()
        plain_norm = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in plain.values())).item()
        # (1) the branches that differ are x3 roundings of 0
        qg, z1, _ = _torch_q_gated(params, X, g1, g2)
        with torch.no_grad():
            z2p = F.linear(F.relu(z1) * m1.float() / 0.8, params["fc2.weight"], params["fc2.bias"])  # torch's fc2
            f1, f2 = ((z1 > 0) & m1.bool()) != g1.bool(), (z2p > 0) != g2.bool()
            n_flips += int(f1.sum()) + int(f2.sum())
            assert int(f1.sum()) <= 1e-5 * f1.numel() and int(f2.sum()) <= 1e-5 * f2.numel(), (int(f1.sum()),
                                                                                              int(f2.sum()))
            if f1.any():
                assert z1[f1].abs().max().item() <= 1e-4 * z1.abs().max().item()
            if f2.any():
                assert z2p[f2].abs().max().item() <= 1e-4 * z2p.abs().max().item()
        # (2) gradients / norm / Adam through the device's branches
        ref_loss = F.mse_loss(qg.gather(1, a.long().unsqueeze(1)).squeeze(), y)
        opt.zero_grad()
        ref_loss.backward()
        gnorm = torch.nn.utils.clip_grad_norm_(params.values(), 1.0)
        grads_ref = {k: p.grad.clone() for k, p in params.items()}
        opt.step()
        torch.cuda.synchronize()
        assert abs(loss.item() - ref_loss.item()) <= 2e-4 * abs(ref_loss.item()) + 1e-5, (it, loss.item(),
                                                                                         ref_loss.item())
        assert abs(loss.item() - F.mse_loss(q_plain.squeeze(), y).item()) <= 2e-4 * abs(loss.item())
        assert abs(lr.norm.item() - gnorm.item()) <= 2e-4 * gnorm.item() + 1e-6, (it, lr.norm.item(), gnorm.item())
        assert abs(lr.norm.item() - plain_norm) <= 1e-3 * plain_norm, (it, lr.norm.item(), plain_norm)
        for k in params:
            ref = grads_ref[k]
            torch.testing.assert_close(lr.grads[k], ref, rtol=2e-3, atol=1e-5 * ref.abs().max().item() + 1e-9,
                                       msg=lambda m: f"B={B} table={table} step {it} grad {k}: {m}")
            diff = (lr.online[k] - params[k].detach()).abs()
            assert (diff > 1e-5).float().mean().item() <= 1e-3, (it, k, diff.max().item())
            assert diff.max().item() <= 2e-3, (it, k, diff.max().item())
    print(f"B={B} table={table}: {n_flips} activations on the other ReLU branch than fp32 torch (x3 roundings of 0)")


def _torch_conv_gated(sd, x, gates, g1, g2):
    """DQNNetwork (agents/dqn_agent.py:15-61, conv variant) with every ReLU / dropout branch
    given: gates[li] = conv layer li's output > 0 on the device (pixel-major [B*121][C]), g1 = keep
    AND fc1 > 0, g2 = fc2 > 0 -- autograd then walks the branches the device's backward walked."""
    B = x.shape[0]
    h = x.permute(0, 3, 1, 2)
    zs = []
    for li, c in enumerate(("conv1", "conv2", "conv3")):
        z = F.conv2d(h, sd[c + ".weight"], sd[c + ".bias"], padding=1)
        zs.append(z)
        gate = gates[li].view(B, 11, 11, -1).permute(0, 3, 1, 2)
        h = z * gate
    z1 = F.linear(h.reshape(B, -1), sd["fc1.weight"], sd["fc1.bias"])
    z2 = F.linear(z1 * g1 / 0.8, sd["fc2.weight"], sd["fc2.bias"])
    return F.linear(z2 * g2, sd["fc3.weight"], sd["fc3.bias"]), zs, z1, z2


def _torch_conv_plain(sd, x, mask):
    B = x.shape[0]
    h = x.permute(0, 3, 1, 2)
    for c in ("conv1", "conv2", "conv3"):
        h = F.relu(F.conv2d(h, sd[c + ".weight"], sd[c + ".bias"], padding=1))
    h = F.relu(F.linear(h.reshape(B, -1), sd["fc1.weight"], sd["fc1.bias"])) * mask.float() / 0.8
    h = F.relu(F.linear(h, sd["fc2.weight"], sd["fc2.bias"]))
    return F.linear(h, sd["fc3.weight"], sd["fc3.bias"])


def test_conv_x3_learn_at_cfg4_batch():
    """Two conv-net learn steps at cfg4's learn batch B = 1024 (the x3 implicit-GEMM convolutions,
    fc1 over K = 15 488 in 16 split-K slices reduced in slice order) from the same parameters and
    Adam moments on both sides, observations of a 256x256 env 30 steps into its episode.
    ReLU branches as test_x3_learn_at_bench_batch: (1) the device's branch differs from torch
    fp32's only where torch's pre-activation is within 1e-4 of the layer's max |z| (the x3
    rounding of 0), on at most 1e-4 of the activations; (2) gradients, norm, loss and the Adam
    update against torch autograd through the DEVICE's branch pattern with the x3 conv bars
    (tests/test_qnet_gpu.py: gradients rtol 2e-3 / atol 1e-3 of max |grad|); (3) loss and norm
    against plain torch. Reference: agents/dqn_agent.py:126-168."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qnet import Learner
    B, R, P = 1024, 1, 9102
    E = 2 * B
    lay = DeviceLayout(build_tables(synthetic(256, 256, R)), P)
    env = VecEnv(lay, E)
    env.seed([700 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(2)
    for _ in range(30):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    torch.cuda.synchronize()
    lr = Learner(kind="conv", precision="x3", seed=43, lr=1e-3)
    sd0 = {k: v.detach().cpu().clone() for k, v in lr.online.state_dict().items()}
    params = {k: torch.nn.Parameter(v.clone()) for k, v in sd0.items()}
    tgt = {k: v.clone() for k, v in sd0.items()}
    opt = torch.optim.Adam(params.values(), lr=1e-3)
    gh = torch.Generator().manual_seed(B)
    xall = env.expand_obs(torch.float32).reshape(E * R, 11, 11, 6).cpu()
    for it in range(2):
        if it > 0:
            lr.online.load_state_dict({k: p.detach().cuda() for k, p in params.items()})
            for key, buf in (("exp_avg", lr.m), ("exp_avg_sq", lr.v)):
                buf.copy_(torch.cat([opt.state[p][key].reshape(-1) for p in params.values()]).cuda())
        perm = torch.randperm(E * R, generator=gh)
        x, x2 = xall[perm[:B]].contiguous(), xall[perm[B:2 * B]].contiguous()
        a = torch.randint(0, 5, (B,), generator=gh, dtype=torch.int32)
        r = torch.randn(B, generator=gh) * 30
        d = (torch.rand(B, generator=gh) < 0.05).to(torch.uint8)
        m1 = (torch.rand(B, 512, generator=gh) >= 0.2).to(torch.uint8)
        m2 = (torch.rand(B, 512, generator=gh) >= 0.2).to(torch.uint8)
        loss = lr.learn(x.cuda(), a.cuda(), r.cuda(), d.cuda(), x2.cuda(), m1.cuda(), m2.cuda())
        torch.cuda.synchronize()
        sv = lr.net.saved
        gates = [(y > 0).float().cpu() for y in sv["ys"]]
        g1, g2 = (sv["H1"] > 0).float().cpu(), (sv["H2"] > 0).float().cpu()
        with torch.no_grad():
            y = r + 0.99 * _torch_conv_plain(tgt, x2, m2).max(1)[0] * (~d.bool())
            plain = {k: p.detach().clone().requires_grad_(True) for k, p in params.items()}
        q_plain = _torch_conv_plain(plain, x, m1).gather(1, a.long().unsqueeze(1))
        plain_loss = F.mse_loss(q_plain.squeeze(), y)
        plain_loss.backward()
        plain_norm = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in plain.values())).item()
        qg, zs, z1, z2 = _torch_conv_gated(params, x, gates, g1, g2)
        with torch.no_grad():  # (1) torch's own branches vs the device's
            h = x.permute(0, 3, 1, 2)
            for li, c in enumerate(("conv1", "conv2", "conv3")):
                z = F.conv2d(h, params[c + ".weight"], params[c + ".bias"], padding=1)
                dev_gate = gates[li].view(B, 11, 11, -1).permute(0, 3, 1, 2).bool()
                f = (z > 0) != dev_gate
                assert int(f.sum()) <= 1e-4 * f.numel(), (c, int(f.sum()))
                if f.any():
                    assert z[f].abs().max().item() <= 1e-4 * z.abs().max().item(), c
                h = F.relu(z)
            z1p = F.linear(h.reshape(B, -1), params["fc1.weight"], params["fc1.bias"])
            f1 = ((z1p > 0) & m1.bool()) != g1.bool()
            assert int(f1.sum()) <= 1e-4 * f1.numel(), int(f1.sum())
            if f1.any():
                assert z1p[f1].abs().max().item() <= 1e-4 * z1p.abs().max().item()
        ref_loss = F.mse_loss(qg.gather(1, a.long().unsqueeze(1)).squeeze(), y)
        opt.zero_grad()
        ref_loss.backward()
        gnorm = torch.nn.utils.clip_grad_norm_(params.values(), 1.0)
        grads_ref = {k: p.grad.clone() for k, p in params.items()}
        opt.step()
        assert abs(loss.item() - ref_loss.item()) <= 2e-4 * abs(ref_loss.item()) + 1e-5, (it, loss.item())
        assert abs(loss.item() - plain_loss.item()) <= 2e-4 * abs(loss.item()) + 1e-5
        assert abs(lr.norm.item() - gnorm.item()) <= 2e-4 * gnorm.item() + 1e-6, (it, lr.norm.item(), gnorm.item())
        assert abs(lr.norm.item() - plain_norm) <= 1e-3 * plain_norm, (it, lr.norm.item(), plain_norm)
        for k in params:
            ref = grads_ref[k]
            torch.testing.assert_close(lr.grads[k].cpu(), ref, rtol=2e-3, atol=1e-3 * ref.abs().max().item() + 1e-9,
                                       msg=lambda m: f"step {it} grad {k}: {m}")
            diff = (lr.online[k].cpu() - params[k].detach()).abs()
            assert (diff > 1e-5).float().mean().item() <= 2e-3, (it, k, diff.max().item())
            assert diff.max().item() <= 1e-3 * 3.3, (it, k, diff.max().item())
