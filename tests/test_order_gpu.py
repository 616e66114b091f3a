"""The two scheduling permutations the training step computes on its side stream, against
numpy restatements on the same state words (evx_state.scal: fire step at [4e], persons
evacuated / dead at [4e + 2] / [4e + 3]):

  * evx_act_perm (act_perm_kernel): the stable partition of the envs by fire step >= t_max
    (the x3 act's table rows first), chunked ballot ranks, one pass per 32768 envs;
  * evx_env_order (env_order32_kernel up to 32768 envs, env_order_kernel beyond): the stable
    counting sort by 16 buckets of persons remaining, heaviest first, and order[E] = the heavy
    count min(176, #envs with >= P/4 persons remaining).

Sizes: ragged (1000), the cfg3 share (32768, one full pass) and 40000 (two act_perm passes, the
slice-per-wave order kernel). Scheduling only -- the env results never depend on these -- but a
wrong permutation would drop or repeat envs."""
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
    perm = torch.full((E + 5,), -7, dtype=torch.int32, device="cuda")
    env.act_perm(perm)
    env.compute_order(force=True)
    torch.cuda.synchronize()
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
