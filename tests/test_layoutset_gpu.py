"""Per-env layouts: one VecEnv over a LayoutSet of three layouts of
one size (different barriers, exits, fire sources), every env bit-exact against the
oracle on its own layout through fused resets; the observations carry the layout and
the MLP fast path reads each row's own static features (vs the plain PyTorch fp32
forward on the expanded reference tensor, tolerances of tests/test_qmlp_gpu.py)."""
import dataclasses

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_env_gpu import gpu_state_fields

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _specs():
    from evacx.layout import synthetic
    s0 = synthetic(24, 20, 4)  # robots start at (10,2) (13,7) (16,12) (20,18)
    s1 = dataclasses.replace(s0, barriers=(((5, 5), (8, 9)),), exit=(24, 3))
    s2 = dataclasses.replace(s0, barriers=(((3, 10), (6, 15)), ((21, 2), (22, 6))), exit=(10, 20),
                             additional_fire=())
    return [s0, s1, s2]


def _setup(E, P=380):
    from evacx.env import DeviceLayout, LayoutSet, VecEnv
    from evacx.layout import build_tables
    tabs = [build_tables(s) for s in _specs()]
    ls = LayoutSet([DeviceLayout(t, P) for t in tabs])
    layout_of = [(i * 7) % 3 for i in range(E)]
    env = VecEnv(ls, E, layout_of=layout_of)
    return tabs, ls, env, layout_of


def test_layout_set_envs_match_oracle_per_layout():
    _need_gpu()
    from oracle import oracle as orc
    P, E = 380, 12
    tabs, ls, env, layout_of = _setup(E, P)
    assert len({float(t.floor[np.isfinite(t.floor)].sum()) for t in tabs}) == 3  # three different floor fields
    R = ls.R
    env.seed([500 + i for i in range(E)])
    olays = [orc.Layout.from_tables(t, P) for t in tabs]
    oenvs = [orc.Env(olays[layout_of[i]]) for i in range(E)]
    for i, oe in enumerate(oenvs):
        oe.seed(500 + i)
    env.reset()
    oobs = [oe.reset() for oe in oenvs]
    rng = np.random.RandomState(3)
    n_done = 0
    for s in range(1, 161):
        acts = rng.randint(0, 5, size=(E, R)).astype(np.int32)
        env.step(torch.from_numpy(acts.reshape(-1)).cuda(), auto_reset=True)
        res = [oe.step(acts[i]) for i, oe in enumerate(oenvs)]
        oobs = [r[0] for r in res]
        rew = env.reward.cpu().numpy()
        done = env.done.cpu().numpy().astype(bool)
        for i in range(E):
            assert rew[i] == res[i][1], (s, i)
            assert done[i] == res[i][2], (s, i)
        if done.any():
            term = env.expand_obs(torch.float64, env.obs_term).cpu().numpy()
            for i in np.nonzero(done)[0]:
                assert np.array_equal(term[i], oobs[i]), (s, i, "terminal obs")
                oobs[i] = oenvs[i].reset()
                n_done += 1
        if s % 20 == 0:
            obs64 = env.expand_obs(torch.float64).cpu().numpy()
            for i in range(E):
                f, st = gpu_state_fields(env, i, obs64)
                ost = oenvs[i].state()
                for name in ["pos", "health", "acc", "flags", "rmap", "robots", "view"]:
                    assert np.array_equal(f[name], ost[name]), (s, i, name)
                assert np.array_equal(st["scal"], ost["scal"]), (s, i)
                assert np.array_equal(st["py_mt"], ost["py_mt"]) and np.array_equal(st["np_mt"], ost["np_mt"])
                assert np.array_equal(obs64[i], oobs[i]), (s, i, "obs")
    env.check_err()
    lid = env.obs.view(E, R, 8)[:, :, 7].cpu().numpy()
    assert (lid == np.asarray(layout_of)[:, None]).all()
    assert n_done > 0


def test_layout_set_mlp_forward_reads_each_rows_layout():
    _need_gpu()
    from evacx.qmlp import HID, K1, MLPFast
    from evacx.qnet import Learner
    E = 48
    tabs, ls, env, layout_of = _setup(E)
    env.seed([900 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(5):
        env.step(torch.randint(0, 5, (E * ls.R,), device="cuda", dtype=torch.int32, generator=g))
    n = E * ls.R
    lr = Learner(kind="mlp", precision="bf16", seed=13)
    fast = MLPFast(lr.online, "cuda")
    h1 = torch.empty(n * HID, dtype=torch.int16, device="cuda")
    q = torch.empty(n, 5, device="cuda")
    fast.forward(ls.c, env.obs, n, h1, q=q)
    torch.cuda.synchronize()
    sd = lr.online.state_dict()
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    X = bf(env.expand_obs(torch.float32).reshape(n, K1))
    z1 = X @ bf(sd["fc1.weight"]).t() + sd["fc1.bias"]
    h = bf(F.relu(z1))
    h2 = F.relu(h @ bf(sd["fc2.weight"]).t() + sd["fc2.bias"])
    qref = h2 @ sd["fc3.weight"].t() + sd["fc3.bias"]
    torch.testing.assert_close(q, qref, rtol=1e-3, atol=1e-3)
    # the per-layout channels really differ: the same window centre reads other barrier /
    # exit / danger features under another layout
    ob = env.obs.view(n, 8).clone()
    ob[:, 7] = (ob[:, 7] + 1) % 3
    q2 = torch.empty(n, 5, device="cuda")
    fast.forward(ls.c, ob.view(-1), n, h1, q=q2)
    X2 = bf(env.expand_obs(torch.float32, ob.view(-1)).reshape(n, K1))
    assert not torch.equal(X2, X)
    h = bf(F.relu(X2 @ bf(sd["fc1.weight"]).t() + sd["fc1.bias"]))
    qref2 = F.relu(h @ bf(sd["fc2.weight"]).t() + sd["fc2.bias"]) @ sd["fc3.weight"].t() + sd["fc3.bias"]
    torch.cuda.synchronize()
    torch.testing.assert_close(q2, qref2, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("lagged", [False, True])
def test_vec_trainer_on_a_layout_set(lagged):
    """The training step over envs of three layouts: it trains (finite losses), and the
    replay's observations carry each env's layout."""
    _need_gpu()
    from evacx.env import DeviceLayout, LayoutSet
    from evacx.layout import build_tables
    from evacx.trainer import VecTrainer
    ls = LayoutSet([DeviceLayout(build_tables(s), 380) for s in _specs()])
    E = 384
    layout_of = [i % 3 for i in range(E)]
    tr = VecTrainer(ls, E, batch=256, replay_capacity=1 << 15, target_every=5, lagged_learn=lagged, lr=1e-3,
                    layout_of=layout_of)
    losses = []
    for _ in range(10):
        tr.step()
        if tr.last_loss is not None:
            losses.append(tr.last_loss)
    tr.sync()
    torch.cuda.synchronize()
    tr.env.check_err()
    assert losses and all(np.isfinite([x.item() for x in losses]))
    n = tr.replay.size
    obs = tr.replay.s.view(-1, 8)[:n].cpu().numpy()
    env_of_row = (np.arange(n) // ls.R) % E
    assert (obs[:, 7] == np.asarray(layout_of)[env_of_row]).all()
