"""The two scheduling permutations the training step computes after every env.step, against
numpy restatements on the same state words (evx_state.scal: fire step at [4e], persons
evacuated / dead at [4e + 2] / [4e + 3]):

  * evx_act_perm: the stable partition of the envs by fire step >= t_max (the x3 act's table
    rows first);
  * evx_env_order: the stable counting sort by 16 buckets of persons remaining, heaviest first,
    and order[E] = the heavy count min(176, #envs with >= P/4 persons remaining);
  * evx_env_orders: both in one launch.
All three read one class byte per env (evx_state.perm_ws), which the step and reset kernels write
as they finish an env (checked against the state words after real steps with auto-resets) and
evx_env_classes rewrites from the state words (here, after scal is written from the host).

Sizes: ragged (1000), the cfg3 share (32768) and 40000. Scheduling only -- the env results never
depend on these -- but a wrong permutation would drop or repeat envs."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _env(E):
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    lay = DeviceLayout(build_tables(synthetic(32, 32, 2)), 200)
    env = VecEnv(lay, E)
    return lay, env


@pytest.mark.parametrize("E", [1000, 32768, 40000])
def test_act_perm_and_env_order_match_numpy(E):
    _need_gpu()
    lay, env = _env(E)
    P, t_max = int(lay.c.P), int(lay.c.t_max)
    rng = np.random.default_rng(E)
    scal = np.zeros((E, 4), np.int32)
    scal[:, 0] = rng.integers(0, t_max + 3, E)        # fire step (some past t_max)
    ev = rng.integers(0, P + 1, E)
    dead = np.minimum(rng.integers(0, P + 1, E), P - ev)
    scal[:, 2] = ev
    scal[:, 3] = dead
    env.scal.view(E, 4).copy_(torch.from_numpy(scal))
    env.refresh_classes()
    perm = torch.full((E + 5,), -7, dtype=torch.int32, device="cuda")
    env.act_perm(perm)
    env.compute_order(force=True)
    perm2 = torch.full((E + 5,), -7, dtype=torch.int32, device="cuda")
    order1 = env.order.clone()
    env.order.fill_(-3)
    env.compute_orders(perm2)  # both in one launch
    torch.cuda.synchronize()
    assert torch.equal(perm, perm2) and torch.equal(order1, env.order)
    sel = scal[:, 0] >= t_max
    want = np.concatenate([np.nonzero(sel)[0], np.nonzero(~sel)[0]]).astype(np.int32)
    got = perm.cpu().numpy()
    assert np.array_equal(got[:E], want)
    assert np.all(got[E:] == -7)
    rem = P - ev - dead
    bucket = 15 - np.minimum(15, np.maximum(0, rem) * 16 // (P + 1))
    want_order = np.argsort(bucket, kind="stable").astype(np.int32)
    order = env.order.cpu().numpy()
    assert np.array_equal(order[:E], want_order)
    assert order[E] == min(176, int(np.sum(rem >= max(1, P // 4))))


def _want_classes(scal, P, t_max):
    rem = P - scal[:, 2] - scal[:, 3]
    b = 15 - np.minimum(15, np.maximum(0, rem) * 16 // (P + 1))
    return (b | np.where(scal[:, 0] >= t_max, 0x10, 0) | np.where(rem >= max(1, P // 4), 0x20, 0)).astype(np.uint8)


def test_step_and_reset_write_class_bytes():
    """The class bytes the step kernel (fused resets included) and the reset kernel leave equal the
    ones the state words give, so the orders after a step need no pass over the state."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    lay = DeviceLayout(build_tables(synthetic(24, 20, 4)), 380)
    E = 700
    env = VecEnv(lay, E)
    env.seed([31 + i for i in range(E)])
    env.reset()
    P, t_max = int(lay.c.P), int(lay.c.t_max)
    g = torch.Generator(device="cuda").manual_seed(2)
    n_done = 0
    for t in range(260):
        env.step(torch.randint(0, 5, (E * lay.R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
        n_done += int(env.done.sum().item())
        if t == 100:
            m = torch.zeros(E, dtype=torch.bool, device="cuda")
            m[::5] = True
            env.reset(mask=m)
        if t % 37 == 0 or t == 101:
            torch.cuda.synchronize()
            scal = env.scal.view(E, 4).cpu().numpy()
            assert np.array_equal(env.perm_ws[:E].cpu().numpy(), _want_classes(scal, P, t_max)), t
    assert n_done > 0


@pytest.mark.parametrize("E", [1000, 32768, 40000])
def test_orders_push_launch_matches_separate_launches(E):
    """evx_env_orders_push_sample (the trainer's one-group step: the replay push, the next orders and
    the learn step's batch in one launch) equals evx_replay_push_term + evx_replay_sample +
    evx_env_orders."""
    _need_gpu()
    from evacx.trainer import Replay
    lay, env = _env(E)
    P, t_max = int(lay.c.P), int(lay.c.t_max)
    rng = np.random.default_rng(E + 1)
    scal = np.zeros((E, 4), np.int32)
    scal[:, 0] = rng.integers(0, t_max + 3, E)
    ev = rng.integers(0, P + 1, E)
    scal[:, 2] = ev
    scal[:, 3] = np.minimum(rng.integers(0, P + 1, E), P - ev)
    env.scal.view(E, 4).copy_(torch.from_numpy(scal))
    env.refresh_classes()
    R = int(lay.c.R)
    n = E * R
    g = torch.Generator(device="cuda").manual_seed(E)
    obs_words = 8
    s = torch.randint(-2**31, 2**31 - 1, (n * obs_words,), device="cuda", dtype=torch.int32, generator=g)
    s2 = torch.randint(-2**31, 2**31 - 1, (n * obs_words,), device="cuda", dtype=torch.int32, generator=g)
    s2t = torch.randint(-2**31, 2**31 - 1, (n * obs_words,), device="cuda", dtype=torch.int32, generator=g)
    a = torch.randint(0, 5, (n,), device="cuda", dtype=torch.int32, generator=g)
    r = torch.randn(E, device="cuda", dtype=torch.float64, generator=g)
    d = (torch.rand(E, device="cuda", generator=g) < 0.3).to(torch.uint8)
    cap = 1 << max(14, (2 * n - 1).bit_length())
    ra, rb = Replay(cap, "cuda"), Replay(cap, "cuda")
    ra.pos = rb.pos = cap - n // 2  # the push wraps around the ring's end
    for rr in (ra, rb):  # older transitions everywhere else in the ring (the same in both)
        rr.s.copy_(torch.arange(rr.s.numel(), device="cuda", dtype=torch.int32))
        rr.s2.copy_(-torch.arange(rr.s2.numel(), device="cuda", dtype=torch.int32))
        rr.a.copy_(torch.arange(cap, device="cuda", dtype=torch.int32) % 5)
        rr.r.copy_(torch.arange(cap, device="cuda", dtype=torch.float32))
        rr.done.copy_((torch.arange(cap, device="cuda") % 3 == 0).to(torch.uint8))
        rr.size = cap - n // 4
    perm1 = torch.full((E + 5,), -7, dtype=torch.int32, device="cuda")
    perm2 = torch.full((E + 5,), -7, dtype=torch.int32, device="cuda")
    B = min(4096, cap // 2)
    out = [dict(s=torch.zeros(B * 8, dtype=torch.int32, device="cuda"),
                s2=torch.zeros(B * 8, dtype=torch.int32, device="cuda"),
                a=torch.zeros(B, dtype=torch.int32, device="cuda"), r=torch.zeros(B, device="cuda"),
                done=torch.zeros(B, dtype=torch.uint8, device="cuda")) for _ in range(2)]
    ra.push(s, s2, a, r, d, n, R, s2_term=s2t)
    ra.sample(B, 77, 12345, out[0])
    env.compute_orders(perm1)
    order1 = env.order.clone()
    env.order.fill_(-3)
    rb.push_orders(env, perm2, s, s2, a, r, d, n, R, s2_term=s2t, sample=(B, 77, 12345, out[1]))  # one launch
    torch.cuda.synchronize()
    assert torch.equal(perm1, perm2) and torch.equal(order1, env.order)
    for name in ("s", "s2", "a", "r", "done"):
        assert torch.equal(getattr(ra, name), getattr(rb, name)), name
        assert torch.equal(out[0][name], out[1][name]), name
    assert (ra.pos, ra.size) == (rb.pos, rb.size)
    # the batch drew slots the push wrote (read from the push's sources) and older ones
    pushed = set(((ra.pos - n + np.arange(n)) % cap).tolist())
    got_r = out[1]["r"].cpu().numpy()
    assert np.any(got_r != np.floor(got_r)) or len(pushed) < cap  # fractional rewards come from the push
