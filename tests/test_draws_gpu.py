"""The GPU's counter-based draws and the composed training step against CPU restatements.

* epsilon-greedy (evx_act, the fused bf16 and x3 act kernels) == oracle.epsilon_greedy of
  the kernel's own Q-values, row for row;
* uniform replay sampling (evx_replay_sample / _window, wrapping windows) == oracle.replay_indices,
  and the gathered rows are the ring's rows at those slots;
* the composed VecTrainer step (strict and lagged): the actions are the epsilon-greedy draw
  of an independent forward with the same weights and dropout stream, and the replay push
  holds (obs before the step, action, team reward, done, obs after the step or the terminal
  obs of an auto-reset env) for every robot."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_evx_act_matches_restatement():
    _need_gpu()
    from evacx.qnet import qcheck, qlib
    g = torch.Generator().manual_seed(1)
    Q = torch.randn(100003, 5, generator=g)
    Q[:100, :] = 1.0  # ties: first maximum
    out = torch.empty(Q.shape[0], dtype=torch.int32, device="cuda")
    for eps, seed, off in [(0.0, 3, 0), (0.3, 5, 12345), (1.0, 9, 2**40 + 7)]:
        qcheck(qlib().evx_act(Q.cuda().data_ptr(), Q.shape[0], 5, eps, seed, off, out.data_ptr(), 0), "act")
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), orc.epsilon_greedy(Q.numpy(), eps, seed, off)), (eps, seed)


@pytest.mark.parametrize("precision", ["bf16", "f32"])
def test_fused_act_epsilon_matches_restatement(precision):
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qnet import Learner
    lay = DeviceLayout(build_tables(synthetic(48, 48, 8)), 300)
    env = VecEnv(lay, 300)
    env.seed(list(range(300)))
    env.reset()
    n = 300 * 8
    lr = Learner(kind="mlp", precision=precision, seed=4)
    q = torch.empty(n, 5, device="cuda")
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    lr.fast.act(lay.c, env.obs, n, drop=(3, 4, 0.2), q=q, actions=a, epsilon=0.4, act_seed=77, act_offset=999)
    torch.cuda.synchronize()
    assert np.array_equal(a.cpu().numpy(), orc.epsilon_greedy(q.cpu().numpy(), 0.4, 77, 999))


@pytest.mark.parametrize("window", [None, (3000, 2000), (100, 3900)])
def test_replay_sampling_matches_restatement(window):
    _need_gpu()
    from evacx.env import OBS_WORDS
    from evacx.qnet import qcheck
    from evacx.trainer import Replay
    import ctypes as C
    from evacx import _lib
    cap = 4096
    B = 4096 if window is None else min(1500, window[1])  # random.sample: B <= population
    rp = Replay(cap, "cuda")
    g = torch.Generator(device="cuda").manual_seed(2)
    rp.s.copy_(torch.randint(-2**31, 2**31 - 1, rp.s.shape, device="cuda", generator=g, dtype=torch.int32))
    rp.s2.copy_(torch.randint(-2**31, 2**31 - 1, rp.s2.shape, device="cuda", generator=g, dtype=torch.int32))
    rp.a.copy_(torch.arange(cap, device="cuda", dtype=torch.int32))
    rp.r.copy_(torch.rand(cap, device="cuda", generator=g))
    rp.done.copy_((torch.rand(cap, device="cuda", generator=g) < 0.5).to(torch.uint8))
    rp.size = cap
    out = dict(s=torch.empty(B * OBS_WORDS, dtype=torch.int32, device="cuda"),
               s2=torch.empty(B * OBS_WORDS, dtype=torch.int32, device="cuda"),
               a=torch.empty(B, dtype=torch.int32, device="cuda"), r=torch.empty(B, device="cuda"),
               done=torch.empty(B, dtype=torch.uint8, device="cuda"))
    idx = torch.empty(B, dtype=torch.int64, device="cuda")
    L = _lib.lib()
    if window is None:
        base, size = 0, cap
        L.evx_replay_sample.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_uint64, C.c_uint64] + [C.c_void_p] * 7
        qcheck(L.evx_replay_sample(C.byref(rp.c), cap, B, 17, 4096, out["s"].data_ptr(), out["s2"].data_ptr(),
                                   out["a"].data_ptr(), out["r"].data_ptr(), out["done"].data_ptr(), idx.data_ptr(),
                                   None), "sample")
    else:
        base, size = window
        L.evx_replay_sample_window.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int32, C.c_uint64,
                                               C.c_uint64] + [C.c_void_p] * 7
        qcheck(L.evx_replay_sample_window(C.byref(rp.c), base, size, B, 17, 4096, out["s"].data_ptr(),
                                          out["s2"].data_ptr(), out["a"].data_ptr(), out["r"].data_ptr(),
                                          out["done"].data_ptr(), idx.data_ptr(), None), "sample_window")
    torch.cuda.synchronize()
    ref = orc.replay_indices(base, size, cap, B, 17, 4096)
    assert np.array_equal(idx.cpu().numpy(), ref)
    assert len(np.unique(ref)) == B  # without replacement
    j = torch.from_numpy(ref).cuda()
    assert torch.equal(out["a"], rp.a[j]) and torch.equal(out["r"], rp.r[j]) and torch.equal(out["done"], rp.done[j])
    assert torch.equal(out["s"].view(B, OBS_WORDS), rp.s.view(cap, OBS_WORDS)[j])
    assert torch.equal(out["s2"].view(B, OBS_WORDS), rp.s2.view(cap, OBS_WORDS)[j])
    if window is None:  # random.sample raises for a sample larger than the population
        assert L.evx_replay_sample(C.byref(rp.c), cap, cap + 1, 17, 0, out["s"].data_ptr(), out["s2"].data_ptr(),
                                   out["a"].data_ptr(), out["r"].data_ptr(), out["done"].data_ptr(), None,
                                   None) != 0


def test_per_agent_replay_sampling_matches_restatement():
    """evx_replay_sample_agents (one memory per robot): agent g's draws are the uniform
    sampler's restated draws (the permutation keyed by stream g) over its own slots (== g mod nets)."""
    _need_gpu()
    from evacx.env import OBS_WORDS
    from evacx.qnet import qcheck
    from evacx.trainer import Replay
    import ctypes as C
    from evacx import _lib
    cap, nets, B, size = 4096, 8, 300, 3000 // 8 * 8
    rp = Replay(cap, "cuda")
    rp.a.copy_(torch.arange(cap, device="cuda", dtype=torch.int32))
    rp.s.copy_(torch.arange(cap * OBS_WORDS, device="cuda", dtype=torch.int32))
    out = dict(s=torch.empty(nets * B * OBS_WORDS, dtype=torch.int32, device="cuda"),
               s2=torch.empty(nets * B * OBS_WORDS, dtype=torch.int32, device="cuda"),
               a=torch.empty(nets * B, dtype=torch.int32, device="cuda"), r=torch.empty(nets * B, device="cuda"),
               done=torch.empty(nets * B, dtype=torch.uint8, device="cuda"))
    L = _lib.lib()
    L.evx_replay_sample_agents.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_uint64,
                                           C.c_uint64] + [C.c_void_p] * 6
    qcheck(L.evx_replay_sample_agents(C.byref(rp.c), size, B, nets, 17, 4096, out["s"].data_ptr(), out["s2"].data_ptr(),
                                      out["a"].data_ptr(), out["r"].data_ptr(), out["done"].data_ptr(), None),
           "sample_agents")
    torch.cuda.synchronize()
    a = out["a"].cpu().numpy().reshape(nets, B)
    for g in range(nets):
        ref = orc.replay_indices(0, size // nets, 1 << 40, B, 17, 4096, stream=g) * nets + g
        assert np.array_equal(a[g], ref), g
    assert torch.equal(out["s"].view(nets * B, OBS_WORDS), rp.s.view(cap, OBS_WORDS)[out["a"].long()])
    assert a.max() < size
    # joint draws (QMIX's memory of env-steps): draw i picks the same env-step for every agent
    L.evx_replay_sample_joint.argtypes = L.evx_replay_sample_agents.argtypes
    qcheck(L.evx_replay_sample_joint(C.byref(rp.c), size, B, nets, 17, 4096, out["s"].data_ptr(), out["s2"].data_ptr(),
                                     out["a"].data_ptr(), out["r"].data_ptr(), out["done"].data_ptr(), None),
           "sample_joint")
    torch.cuda.synchronize()
    aj = out["a"].cpu().numpy().reshape(nets, B)
    step = orc.replay_indices(0, size // nets, 1 << 40, B, 17, 4096)
    for g in range(nets):
        assert np.array_equal(aj[g], step * nets + g), g
    assert L.evx_replay_sample_agents(C.byref(rp.c), size + 1, B, nets, 17, 0, out["s"].data_ptr(),
                                      out["s2"].data_ptr(), out["a"].data_ptr(), out["r"].data_ptr(),
                                      out["done"].data_ptr(), None) != 0  # size not a multiple of nets


@pytest.mark.parametrize("mode", ["strict", "lagged"])
def test_trainer_step_composition(mode):
    _need_gpu()
    from evacx.env import OBS_WORDS, DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.qmlp import HID
    from evacx.qnet import DROPOUT_P
    from evacx.trainer import VecTrainer
    E, R = 96, 4
    lay = DeviceLayout(build_tables(synthetic(32, 32, R)), 120)
    lagged = mode == "lagged"
    tr = VecTrainer(lay, E, batch=128, replay_capacity=8192, lagged_learn=lagged, epsilon=0.5)
    env, n = tr.env, E * R
    checked_done = 0
    for t in range(12):
        tr.sync()
        torch.cuda.synchronize()
        obs0 = env.obs.clone()
        eps, off, stream = tr.epsilon, tr.t * tr.n_world + tr.agent0, tr.learner.drop_stream + 1
        h1 = torch.empty(2 * n * HID, dtype=torch.int16, device="cuda")
        q = torch.empty(n, 5, device="cuda")
        tr.fast.forward(lay.c, obs0, n, h1, drop=(tr.learner.seed, stream, DROPOUT_P, None, tr.agent0), q=q)
        pos0 = tr.replay.pos
        tr.step()
        tr.sync()
        torch.cuda.synchronize()
        acts = tr.actions.cpu().numpy()
        assert np.array_equal(acts, orc.epsilon_greedy(q.cpu().numpy(), eps, tr.act_seed, off)), t
        sl = slice(pos0, pos0 + n)
        rp = tr.replay
        done = env.done.cpu().numpy().astype(bool)
        assert torch.equal(rp.s.view(-1, OBS_WORDS)[sl], obs0.view(-1, OBS_WORDS))
        assert np.array_equal(rp.a[sl].cpu().numpy(), acts)
        assert np.array_equal(rp.r[sl].cpu().numpy(), np.repeat(env.reward.cpu().numpy().astype(np.float32), R))
        assert np.array_equal(rp.done[sl].cpu().numpy().astype(bool), np.repeat(done, R))
        s2 = torch.where(torch.from_numpy(np.repeat(done, R)).cuda()[:, None], env.obs_term.view(-1, OBS_WORDS),
                         env.obs.view(-1, OBS_WORDS))
        assert torch.equal(rp.s2.view(-1, OBS_WORDS)[sl], s2)
        checked_done += int(done.sum())
    assert tr.learn_steps >= 10 and np.isfinite(tr.last_loss.item())
