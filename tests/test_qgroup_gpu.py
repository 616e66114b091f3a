"""GPU parity of the grouped independent nets (evacx.qgroup, SURVEY §8f F3: one network per robot
as runners/train_double_dqn.py:35-56 trains them, and the QMIX mixer of runners/train_qmix.py:39-118).

* grouped learn == G separate evacx.qnet.Learner steps (same initial weights, same dropout
  keys): losses, norms, clipped gradients, parameters and Adam state within the run-to-run ulps
  of the f32 atomic sums both paths use for the small gradients (fc3, fc2.bias, fc1.bias);
* grouped act == the single-net act per robot (Q bit for bit, dropout keyed by the net's own
  batch rows) and epsilon draws keyed by the data row as the shared-net act;
* evx_qmix_loss (mixer forward, MSE, backward into every agent's dQ, mixer gradient) vs torch
  autograd of MixingNetwork (f32 tolerance: different summation order);
* GroupedQMix's learn steps vs torch fp32 autograd of the agents and MixingNetwork (loss,
  clipped gradients, agent and mixer parameters after Adam).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _env_obs(E=96, steps=5, R=4, grid=48, people=300):
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    lay = DeviceLayout(build_tables(synthetic(grid, grid, R)), people)
    env = VecEnv(lay, E)
    env.seed([91 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(steps):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g))
    torch.cuda.synchronize()
    return lay, env


def _batch(env, G, B, g):
    obs = env.obs.view(-1, 8)
    n = obs.shape[0]
    s = obs[torch.randint(0, n, (G * B,), generator=g).cuda()].contiguous().view(-1)
    s2 = obs[torch.randint(0, n, (G * B,), generator=g).cuda()].contiguous().view(-1)
    a = torch.randint(0, 5, (G * B,), generator=g, dtype=torch.int32).cuda()
    r = (torch.randn(G * B, generator=g) * 30).cuda()
    d = (torch.rand(G * B, generator=g) < 0.2).to(torch.uint8).cuda()
    return s, s2, a, r, d


@pytest.mark.parametrize("G,B", [(3, 256), (2, 190)])
def test_grouped_learn_equals_separate_learners(G, B):
    _need_gpu()
    from evacx.qgroup import GroupedLearner
    from evacx.qnet import Learner
    lay, env = _env_obs()
    grp = GroupedLearner(G, seed=40, lr=1e-3)
    sep = []
    for k in range(G):
        lr = Learner(kind="mlp", precision="f32", seed=40 + k, lr=1e-3)
        lr.seed = grp.seed  # the dropout hash seed; rows keyed k * B + i below
        sep.append(lr)
        assert torch.equal(lr.online.flat, grp.flat[k])
    g = torch.Generator().manual_seed(5)
    for it in range(3):
        s, s2, a, r, d = _batch(env, G, B, g)
        loss = grp.learn_obs(lay.c, s, a, r, d, s2, B).clone()
        for k, lr in enumerate(sep):
            rows = slice(k * B, (k + 1) * B)
            lk = lr.learn_obs(lay.c, s.view(-1, 8)[rows].contiguous().view(-1), a[rows].contiguous(),
                              r[rows].contiguous(), d[rows].contiguous(), s2.view(-1, 8)[rows].contiguous().view(-1),
                              B, drop_row0=k * B)
            torch.cuda.synchronize()
            # the small gradients (fc3, fc2.bias, fc1.bias and W1's centre column) are f32 atomic
            # sums in both paths (order varies run to run, ulps); the rest is bit-deterministic
            assert abs(loss[k].item() - lk.item()) <= 1e-6 * abs(lk.item()), (it, k, loss[k].item(), lk.item())
            assert abs(grp.norm[k].item() - lr.norm.item()) <= 1e-6 * lr.norm.item(), (it, k)
            torch.testing.assert_close(grp.gflat[k], lr.grads.flat, rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(grp.flat[k], lr.online.flat, rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(grp.m[k], lr.m, rtol=1e-5, atol=1e-8)
            torch.testing.assert_close(grp.v[k], lr.v, rtol=1e-4, atol=1e-12)
            for name in ("w1b", "w2b", "w2t", "w1o"):  # bf16 hi operand copies of the params (lo: residual ulps)
                same = (grp.fast.bufs[name][k] == getattr(lr.fast, name)).float().mean().item()
                assert same >= 0.999, (it, k, name, same)
        if it == 1:
            grp.sync_target()
            for lr in sep:
                lr.sync_target()
    assert len({round(float(x), 3) for x in loss}) == G  # the nets really differ


@pytest.mark.parametrize("eps", [0.0, 1.0])
def test_grouped_act_equals_single_net_act(eps):
    _need_gpu()
    from evacx.qgroup import GroupedLearner
    from evacx.qmlp import NACT
    R = 4
    lay, env = _env_obs(E=300, R=R)
    E = env.E
    grp = GroupedLearner(R, seed=8)
    q = torch.full((E * R, NACT), 7.0, device="cuda")
    act = torch.full((E * R,), -1, dtype=torch.int32, device="cuda")
    grp.act(lay.c, env.obs, E, actions=act, q=q, epsilon=eps, act_seed=9, act_offset=33, drop_stream=12)
    obs = env.obs.view(E, R, 8)
    for k in range(R):
        ok = obs[:, k].contiguous().view(-1)
        qk = torch.empty(E, NACT, device="cuda")
        ak = torch.empty(E, dtype=torch.int32, device="cuda")
        grp.fast.nets[k].act(lay.c, ok, E, drop=(grp.seed, 12, 0.2, None, k * E), q=qk, actions=ak)
        torch.cuda.synchronize()
        assert torch.equal(q.view(E, R, NACT)[:, k], qk), k
        if eps == 0.0:
            assert torch.equal(act.view(E, R)[:, k], ak), k
    if eps == 1.0:  # every action drawn: keyed by the data row (env * R + robot), as the shared-net act
        ref = torch.empty(E * R, dtype=torch.int32, device="cuda")
        grp.fast.nets[0].act(lay.c, env.obs, E * R, drop=(grp.seed, 12, 0.2), actions=ref, epsilon=1.0, act_seed=9,
                             act_offset=33)
        torch.cuda.synchronize()
        assert torch.equal(act, ref)


def test_qmix_kernel_matches_torch_autograd():
    _need_gpu()
    from evacx.qmix import MixingNetwork
    from evacx.qmlp import mlib
    n, B, A = 3, 700, 5
    torch.manual_seed(2)
    mix, mix_t = MixingNetwork(n).cuda(), MixingNetwork(n).cuda()
    with torch.no_grad():
        mix.fc1_bias.normal_()
        mix.fc2_bias.normal_()
        mix.fc1_weight[0, 3] = 0.0  # sign(0) = 0 in torch.abs' gradient
    Q = torch.randn(n, B, A, device="cuda") * 5
    Qt = torch.randn(n, B, A, device="cuda") * 5
    act = torch.randint(0, A, (n, B), device="cuda", dtype=torch.int32)
    rew = torch.randn(B, device="cuda") * 10
    done = (torch.rand(B, device="cuda") < 0.3).to(torch.uint8)
    flat = torch.cat([p.detach().reshape(-1) for p in mix.state_dict().values()])
    flat_t = torch.cat([p.detach().reshape(-1) for p in mix_t.state_dict().values()])
    nm = int(mlib().evx_qmix_nparams(n))
    assert nm == flat.numel()
    dQ = torch.full((n, B, A), 5.0, device="cuda")
    grad = torch.empty(nm, device="cuda")
    loss = torch.empty(1, device="cuda")
    part = torch.empty(int(mlib().evx_qmix_part_floats(B, n)), device="cuda")
    zero = torch.ones(1000, device="cuda")
    rc = mlib().evx_qmix_loss(Q.data_ptr(), Qt.data_ptr(), A, act.data_ptr(), rew.data_ptr(), done.data_ptr(), 0.99, B,
                              n, flat.data_ptr(), flat_t.data_ptr(), dQ.data_ptr(), grad.data_ptr(), loss.data_ptr(),
                              part.data_ptr(), zero.data_ptr(), zero.numel(), None)
    assert rc == 0
    q = Q.gather(2, act.long().unsqueeze(2)).squeeze(2).t().contiguous().requires_grad_(True)  # [B][n]
    with torch.no_grad():
        y = rew + 0.99 * mix_t(Qt.max(2)[0].t()) * (~done.bool()).float()
    ref = torch.nn.functional.mse_loss(mix(q), y)
    mix.zero_grad()
    ref.backward()
    torch.cuda.synchronize()
    assert torch.count_nonzero(zero) == 0
    torch.testing.assert_close(loss[0], ref.detach(), rtol=1e-5, atol=1e-6)
    gref = torch.cat([p.grad.reshape(-1) for p in mix.parameters()])
    torch.testing.assert_close(grad, gref, rtol=1e-4, atol=1e-5 * gref.abs().max().item())
    assert grad[3].item() == 0.0
    dref = torch.zeros(n, B, A, device="cuda")
    dref.scatter_(2, act.long().unsqueeze(2), q.grad.t().unsqueeze(2))
    torch.testing.assert_close(dQ, dref, rtol=1e-4, atol=1e-6 * dref.abs().max().item())


def test_grouped_qmix_step_matches_torch_autograd():
    """Two QMIX learn steps (runners/train_qmix.py:78-113) from the same state: GroupedQMix
    (grouped x3 kernels + evx_qmix_loss + per-agent clip/Adam + mixer clip/Adam) vs torch fp32
    autograd of the agents' fc stacks and MixingNetwork on the expanded observations, dropout off
    on both sides (p = 0): loss, clipped agent gradients, agent parameters, mixer parameters."""
    _need_gpu()
    import torch.nn.functional as F
    from evacx.qgroup import GroupedLearner, GroupedQMix
    from evacx.qmix import MixingNetwork
    from evacx.qmlp import K1
    n, B = 2, 128
    lay, env = _env_obs(R=2)
    grp = GroupedLearner(n, seed=60, lr=1e-3)
    grp.drop_p = 0.0
    torch.manual_seed(3)
    mixing, target_mixing = MixingNetwork(n).cuda(), MixingNetwork(n).cuda()
    target_mixing.load_state_dict(mixing.state_dict())
    qm = GroupedQMix(grp, mixing=mixing)
    agents = [{k: torch.nn.Parameter(v.clone()) for k, v in grp.online[j].state_dict().items()} for j in range(n)]
    targets = [{k: v.clone() for k, v in grp.target[j].state_dict().items()} for j in range(n)]
    opts = [torch.optim.Adam(p.values(), lr=1e-3) for p in agents]
    mopt = torch.optim.Adam(mixing.parameters(), lr=1e-3)

    def fc(sd, X):
        h = F.relu(F.linear(X, sd["fc1.weight"], sd["fc1.bias"]))
        h = F.relu(F.linear(h, sd["fc2.weight"], sd["fc2.bias"]))
        return F.linear(h, sd["fc3.weight"], sd["fc3.bias"])
    g = torch.Generator().manual_seed(4)
    for it in range(2):
        s, s2, a, _, _ = _batch(env, n, B, g)
        r = (torch.randn(B, generator=g) * 30).cuda()
        d = (torch.rand(B, generator=g) < 0.2).to(torch.uint8).cuda()
        loss = qm(lay.c, s, a, r, d, s2, B)
        X = env.expand_obs(torch.float32, s).reshape(n, B, K1)
        X2 = env.expand_obs(torch.float32, s2).reshape(n, B, K1)
        av = a.view(n, B).long()
        q = torch.stack([fc(agents[j], X[j]).gather(1, av[j].unsqueeze(1)).squeeze(1) for j in range(n)], 1)
        with torch.no_grad():
            qt = torch.stack([fc(targets[j], X2[j]).max(1)[0] for j in range(n)], 1)
            y = r + 0.99 * target_mixing(qt) * (~d.bool())
        ref = F.mse_loss(mixing(q), y)
        for o in opts + [mopt]:
            o.zero_grad()
        ref.backward()
        norms = [torch.nn.utils.clip_grad_norm_(p.values(), 1.0) for p in agents]
        mnorm = torch.nn.utils.clip_grad_norm_(mixing.parameters(), 1.0)
        grads = [torch.cat([p.grad.reshape(-1) for p in ag.values()]) for ag in agents]
        for o in opts + [mopt]:
            o.step()
        torch.cuda.synchronize()
        assert abs(loss.item() - ref.item()) <= 2e-4 * abs(ref.item()) + 1e-5, (it, loss.item(), ref.item())
        for j in range(n):
            assert abs(grp.norm[j].item() - norms[j].item()) <= 2e-4 * norms[j].item() + 1e-6, (it, j)
            # x3 products (~2^-16 relative) under cancellation: a few of 5e5 elements beyond rtol 2e-3
            gs = grads[j].abs().max().item()
            bad = (grp.gflat[j] - grads[j]).abs() > 2e-3 * grads[j].abs() + 1e-5 * gs
            assert bad.float().mean().item() <= 1e-4, (it, j, int(bad.sum()))
            assert (grp.gflat[j] - grads[j]).abs().max().item() <= 1e-3 * gs, (it, j)
            pref = torch.cat([p.detach().reshape(-1) for p in agents[j].values()])
            diff = (grp.flat[j] - pref).abs()
            assert (diff > 1e-5).float().mean().item() <= 1e-3 and diff.max().item() <= 2e-3, (it, j)
        assert abs(qm.mix_norm.item() - mnorm.item()) <= 2e-4 * mnorm.item() + 1e-6
        mref = torch.cat([p.detach().reshape(-1) for p in mixing.state_dict().values()])
        torch.testing.assert_close(qm.mix, mref, rtol=1e-4, atol=1e-5)


def test_vec_trainer_per_robot_nets():
    """VecTrainer(nets="per_robot"): robot r of every env acts through net r (== the grouped act
    on the same observations and weights), every net learns from its own robot's transitions
    (the per-agent sampler) and moves; the shared-net parameters are untouched by construction."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    R, E = 4, 64
    lay = DeviceLayout(build_tables(synthetic(48, 48, R)), 300)
    tr = VecTrainer(lay, E, batch=8 * R * 2, replay_capacity=1 << 12, nets="per_robot", epsilon=0.3, learner_seed=3)
    p0 = tr.glearner.flat.clone()
    for _ in range(6):
        tr.step()
    tr.sync()
    torch.cuda.synchronize()
    assert tr.last_loss is not None and tr.last_loss.shape == (R,) and torch.isfinite(tr.last_loss).all()
    moved = (tr.glearner.flat != p0).any(dim=1)
    assert bool(moved.all())
    # the next act == a grouped act with the trainer's draws
    a_ref = torch.empty(E * R, dtype=torch.int32, device="cuda")
    off = tr.t * tr.n_world + tr.agent0
    stream = 0x40000000 + tr.glearner._act_calls + 1
    tr.glearner.act(lay.c, tr.env.obs, E, actions=a_ref, epsilon=float(tr.epsilon), act_seed=tr.act_seed,
                    act_offset=off, drop_stream=stream)
    a = tr.act()
    torch.cuda.synchronize()
    assert torch.equal(a, a_ref)


def test_vec_trainer_qmix_nets():
    """VecTrainer(nets="qmix"): the robots of an env as the agents of runners/train_qmix.py --
    joint samples, GroupedQMix learn steps (mixer kernel), every agent and the mixer move."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    R, E = 4, 64
    lay = DeviceLayout(build_tables(synthetic(48, 48, R)), 300)
    tr = VecTrainer(lay, E, batch=8 * R * 2, replay_capacity=1 << 12, nets="qmix", epsilon=0.3, learner_seed=5,
                    target_every=3)
    p0, m0 = tr.glearner.flat.clone(), tr.qmix.mix.clone()
    for _ in range(8):
        tr.step()
    tr.sync()
    torch.cuda.synchronize()
    assert tr.last_loss is not None and torch.isfinite(tr.last_loss).all()
    assert bool((tr.glearner.flat != p0).any(dim=1).all()) and not torch.equal(tr.qmix.mix, m0)
    assert torch.equal(tr.qmix.mix_t, tr.qmix.mix) or tr.learn_steps % 3 != 0
