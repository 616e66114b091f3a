"""The device-resident vectorised training loop (evacx.trainer) on the GPU."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("precision", ["bf16", "f32"])
def test_vec_trainer_runs_and_learns(precision):
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    spec = synthetic(64, 64, 4)
    lay = DeviceLayout(build_tables(spec), 300)
    tr = VecTrainer(lay, 64, precision=precision, batch=256, replay_capacity=4096, epsilon_decay=0.99,
                    target_every=5)
    p0 = tr.learner.online.flat.clone()
    losses = []
    for _ in range(20):
        tr.step()
        tr.sync()  # the trainer runs on its own streams
        if tr.last_loss is not None:
            losses.append(tr.last_loss.item())
    tr.env.check_err()
    assert tr.replay.size == min(4096, 20 * 64 * 4)
    assert len(losses) == 20 and all(np.isfinite(losses))
    assert tr.epsilon < 1.0
    assert not torch.equal(p0, tr.learner.online.flat)
    a = tr.actions.cpu().numpy()
    assert a.min() >= 0 and a.max() <= 4
    # replay holds the transitions: actions in range, compact obs centred inside the grid
    obs = tr.replay.s.view(-1, 8)[:tr.replay.size].cpu().numpy()
    assert (obs[:, 4] >= 0).all() and (obs[:, 4] <= 65).all()


def test_replay_push_sample_roundtrip():
    _need_gpu()
    from evacx.trainer import Replay
    rp = Replay(100, torch.device("cuda"))
    n = 30
    s = torch.arange(n * 8, dtype=torch.int32, device="cuda")
    s2 = s + 1000
    a = torch.arange(n, dtype=torch.int32, device="cuda") % 5
    r_env = torch.arange(n // 3, dtype=torch.float64, device="cuda")
    d_env = (torch.arange(n // 3, device="cuda") % 2).to(torch.uint8)
    for _ in range(4):
        rp.push(s, s2, a, r_env, d_env, n, 3)
    assert rp.size == 100 and rp.pos == 20
    out = dict(s=torch.zeros(64 * 8, dtype=torch.int32, device="cuda"),
               s2=torch.zeros(64 * 8, dtype=torch.int32, device="cuda"),
               a=torch.zeros(64, dtype=torch.int32, device="cuda"),
               r=torch.zeros(64, dtype=torch.float32, device="cuda"),
               done=torch.zeros(64, dtype=torch.uint8, device="cuda"))
    rp.sample(64, 5, 0, out)
    so = out["s"].view(64, 8).cpu().numpy()
    i = so[:, 0] // 8  # which agent row each sample came from
    assert np.array_equal(out["s2"].view(64, 8).cpu().numpy()[:, 0], so[:, 0] + 1000)
    assert np.array_equal(out["a"].cpu().numpy(), i % 5)
    assert np.array_equal(out["r"].cpu().numpy(), (i // 3).astype(np.float32))
    assert np.array_equal(out["done"].cpu().numpy(), (i // 3) % 2)


def test_replay_sample_window_stays_inside():
    """evx_replay_sample_window draws only from [base, base+count) mod capacity."""
    _need_gpu()
    from evacx.trainer import Replay
    rp = Replay(100, torch.device("cuda"))
    n = 30
    s = torch.arange(n * 8, dtype=torch.int32, device="cuda")
    z = torch.zeros(n // 3, device="cuda", dtype=torch.float64)
    dz = torch.zeros(n // 3, device="cuda", dtype=torch.uint8)
    for _ in range(4):  # slots 90..99, 0..19 hold the last push; pos = 20
        rp.push(s + 1000 * _, s, torch.zeros(n, dtype=torch.int32, device="cuda"), z, dz, n, 3)
    base, count = rp.window(n)
    assert (base, count) == (50, 70)  # the newest 70 entries (slots 50..99, 0..19); a push of 30 overwrites 20..49
    out = dict(s=torch.zeros(4096 * 8, dtype=torch.int32, device="cuda"),
               s2=torch.zeros(4096 * 8, dtype=torch.int32, device="cuda"),
               a=torch.zeros(4096, dtype=torch.int32, device="cuda"),
               r=torch.zeros(4096, dtype=torch.float32, device="cuda"),
               done=torch.zeros(4096, dtype=torch.uint8, device="cuda"))
    ring = rp.s.view(100, 8)[:, 0].cpu().numpy()
    slot = {int(v): k for k, v in enumerate(ring)}
    # slot k of the ring holds push (k + 4*30 - 20 ...): recover the slots from the stored values
    for off, B in ((0, count), (70, 40), (110, 1)):  # without replacement: B <= count distinct slots
        rp.sample_window(base, count, B, 9, off, out)
        got = out["s"].view(4096, 8)[:B, 0].cpu().numpy()
        slots = np.array([slot[int(v)] for v in got])
        assert ((slots - base) % 100 < count).all()
        assert len(np.unique(slots)) == B  # B = count: every slot of the window exactly once
    with pytest.raises(Exception, match="larger than the window"):
        rp.sample_window(base, count, count + 1, 9, 0, out)


@pytest.mark.parametrize("lagged", [False, True])
def test_vec_trainer_schedules(lagged):
    """strict and lagged-learn schedules both train; the lagged learn overlaps env.step."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    lay = DeviceLayout(build_tables(synthetic(64, 64, 4)), 300)
    tr = VecTrainer(lay, 64, batch=256, replay_capacity=2048, target_every=5, lagged_learn=lagged, lr=1e-3)
    losses = []
    for _ in range(40):
        tr.step()
        if tr.last_loss is not None:
            losses.append(tr.last_loss)
    tr.sync()
    torch.cuda.synchronize()
    tr.env.check_err()
    losses = [x.item() for x in losses]
    assert len(losses) == (40 - 1 if lagged else 40)  # lagged: the first step has an empty ring
    assert all(np.isfinite(losses))
    assert tr.replay.size == 2048


@pytest.mark.parametrize("lagged", [False, True])
def test_vec_trainer_groups(lagged):
    """Two env groups on their own stream chains: the schedule trains (strict and lagged),
    every transition lands in the ring, the env state stays valid."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    lay = DeviceLayout(build_tables(synthetic(24, 20, 4)), 380)
    tr = VecTrainer(lay, 512, batch=256, replay_capacity=1 << 15, target_every=5, lagged_learn=lagged, lr=1e-3,
                    groups=2)
    losses = []
    for _ in range(12):
        tr.step()
        if tr.last_loss is not None:
            losses.append(tr.last_loss)
    tr.sync()
    torch.cuda.synchronize()
    tr.env.check_err()
    assert len(losses) == (11 if lagged else 12) and all(np.isfinite([x.item() for x in losses]))
    assert tr.replay.size == 12 * 512 * 4
    a = tr.replay.a[:tr.replay.size].cpu().numpy()
    assert a.min() >= 0 and a.max() <= 4
    obs = tr.replay.s.view(-1, 8)[:tr.replay.size].cpu().numpy()
    assert (obs[:, 4] >= 0).all() and (obs[:, 4] <= 25).all()


def test_same_seed_trainers_are_bit_identical():
    """Two VecTrainers with the same seeds at cfg3's geometry (128x128, P 2276, R 16; E = 4096,
    learn batch 4096) agree bit for bit after 10 training steps: weights, target weights, Adam
    moments, env state (people, health, rmap, robots, MT19937 streams), actions. DQNAgent.learn
    (agents/dqn_agent.py:126-168) on torch-CPU gives the same weights on every same-seed run; the
    learn chain here sums every gradient through partials in a fixed order (no f32 atomics)."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    lay = DeviceLayout(build_tables(synthetic(128, 128, 16)), 2276)
    snaps = []
    for _ in range(2):
        tr = VecTrainer(lay, 4096, batch=4096, replay_capacity=1 << 20, epsilon=0.3, target_every=4)
        acts = []
        for _ in range(10):
            tr.step()
            with torch.cuda.stream(tr.main):  # the trainer's stream: after this step's act, before the next
                acts.append(tr.actions.clone())
        tr.sync()
        torch.cuda.synchronize()
        tr.env.check_err()
        lr, env = tr.learner, tr.env
        assert tr.learn_steps == 10
        snaps.append(dict(online=lr.online.flat.clone(), target=lr.target.flat.clone(), m=lr.m.clone(),
                          v=lr.v.clone(), loss=tr.last_loss.clone(), pk=env.pk.clone(), health=env.health.clone(),
                          acc=env.acc.clone(), rmap=env.rmap.clone(), robots=env.robots.clone(),
                          scal=env.scal.clone(), py_mt=env.py_mt.clone(), np_mt=env.np_mt.clone(),
                          obs=env.obs.clone(), acts=torch.stack(acts), ring=tr.replay.s.clone()))
        del tr, lr, env
        torch.cuda.empty_cache()
    a, b = snaps
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_groups_match_one_group():
    """VecTrainer(groups=2) -- two stream chains, group 1's act overlapping group 0's env.step --
    against groups=1 from the same seeds (epsilon 1: the actions do not depend on the Q values):
    env states, the replay ring (transitions land in global agent order), the act's dropout stream
    and, through identical learn batches, the online weights are bit-identical after 8 steps."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    lay = DeviceLayout(build_tables(synthetic(128, 128, 16)), 2276)
    snaps = []
    for G in (1, 2):
        tr = VecTrainer(lay, 2048, batch=2048, replay_capacity=1 << 18, epsilon=1.0, epsilon_decay=1.0,
                        target_every=3, groups=G)
        for _ in range(8):
            tr.step()
        tr.sync()
        torch.cuda.synchronize()
        tr.env.check_err()
        env = tr.env
        snaps.append(dict(online=tr.learner.online.flat.clone(), pk=env.pk.clone(), health=env.health.clone(),
                          scal=env.scal.clone(), py_mt=env.py_mt.clone(), np_mt=env.np_mt.clone(),
                          ring=tr.replay.s.clone(), ring_a=tr.replay.a.clone(), ring_r=tr.replay.r.clone(),
                          drop=tr.learner.drop_stream))
        del tr, env
        torch.cuda.empty_cache()
    a, b = snaps
    for k in a:
        assert (a[k] == b[k]) if k == "drop" else torch.equal(a[k], b[k]), k


def test_groups_greedy_act_matches_one_group():
    """The x3 act's table path with per-group env orders (grp.perm, a slice of the trainer's
    permutation, rows_per_env = R) at epsilon 0, so the actions are the argmax of the act's Q:
    every env at the layout's last fire step (every tile takes the table path, where a row's Q
    does not depend on the tile it shares), G = 2 against G = 1 from the same seeds -- the
    greedy actions are identical and depend on the Q values (not all one action). A wrong perm
    slice or row offset in a group would move Q values between robots."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    lay = DeviceLayout(build_tables(synthetic(128, 128, 16)), 2276)
    t_max = int(lay.c.t_max)
    acts = []
    for G in (1, 2):
        tr = VecTrainer(lay, 2048, batch=2048, replay_capacity=1 << 16, epsilon=0.0, epsilon_min=0.0,
                        epsilon_decay=1.0, groups=G)
        env = tr.env
        assert tr.fast is not None
        env.scal.view(env.E, 4)[:, 0] = t_max
        env.obs.view(-1, 8)[:, 6] = t_max
        env.refresh_classes()
        for grp in tr.groups:
            grp.env.compute_orders(perm=grp.perm)
        torch.cuda.synchronize()
        tr.act()
        tr.sync()
        torch.cuda.synchronize()
        acts.append(tr.actions.clone())
        del tr, env
        torch.cuda.empty_cache()
    assert torch.equal(acts[0], acts[1])
    counts = torch.bincount(acts[0].long(), minlength=5)
    assert int((counts > 0).sum()) >= 2, counts


@pytest.mark.gpu
def test_fused_push_orders_sample_matches_separate_launches():
    """The one-group strict step draws its learn batch in the replay push + orders launch
    (evx_env_orders_push_sample). Against the same trainer with that launch disabled (a Replay
    subclass: separate push, orders on the side stream, the sample in learn()) from the same seeds,
    10 steps at cfg3's geometry (E = 4096, B = 4096, capacity 2^17 so the ring wraps): weights, Adam
    moments, the replay ring, the env state and every step's actions are bit-identical."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import Replay, VecTrainer

    class _Separate(Replay):  # type(replay) is not Replay: the trainer takes the separate launches
        pass

    lay = DeviceLayout(build_tables(synthetic(128, 128, 16)), 2276)
    snaps = []
    for separate in (False, True):
        tr = VecTrainer(lay, 4096, batch=4096, replay_capacity=1 << 17, epsilon=0.3, target_every=4)
        drawn = []
        if separate:
            tr.replay.__class__ = _Separate
        else:  # count the fused launches that drew the learn batch
            fused_call = tr.replay.push_orders

            def counted(*args, sample=None, **kw):
                drawn.append(sample is not None)
                return fused_call(*args, sample=sample, **kw)
            tr.replay.push_orders = counted
        acts = []
        for _ in range(10):
            tr.step()
            with torch.cuda.stream(tr.main):
                acts.append(tr.actions.clone())
        tr.sync()
        torch.cuda.synchronize()
        tr.env.check_err()
        assert tr.learn_steps == 10
        assert drawn == ([] if separate else [True] * 10), drawn
        lr, env = tr.learner, tr.env
        snaps.append(dict(online=lr.online.flat.clone(), target=lr.target.flat.clone(), m=lr.m.clone(),
                          v=lr.v.clone(), loss=tr.last_loss.clone(), pk=env.pk.clone(), health=env.health.clone(),
                          rmap=env.rmap.clone(), robots=env.robots.clone(), obs=env.obs.clone(),
                          acts=torch.stack(acts), ring=tr.replay.s.clone(), ring_a=tr.replay.a.clone()))
        del tr, lr, env
        torch.cuda.empty_cache()
    a, b = snaps
    for k in a:
        assert torch.equal(a[k], b[k]), k
