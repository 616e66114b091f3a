"""The x3 act's row order (evx_act_row_perm) and the act through it (qact3h_kernel DM 3).

DQNAgent.act (agents/dqn_agent.py:101-124) for every robot: VecTrainer sorts the act's rows by
(on the act table's path or not, window centre) so rows sharing a table row share 64-row tiles.
The order must change no result: every row's Q, dropout mask (each tile row hashes its own
dropout pair) and epsilon draw stay keyed by the row itself.

* the permutation equals numpy's stable argsort of the same keys (a permutation of every row);
* with every row on the table path (all at the fire's last step), the row-permuted act gives
  the unpermuted act's Q and actions bit for bit (same products, same order per row, same masks);
* with a mixed batch, rows the permutation puts in uniform table tiles equal the unpermuted act
  wherever that act took the same path (compared on the rows of all-table tiles of both), and
  the actions of the whole batch match the oracle's epsilon-greedy rule of the permuted act's Q.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _row_perm(lay, obs, n, fast):
    from evacx import _lib
    L = _lib.lib()
    L.evx_act_row_perm_bytes.restype = C.c_int64
    L.evx_act_row_perm_bytes.argtypes = [C.c_int32]
    L.evx_act_row_perm.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    nb = int(L.evx_act_row_perm_bytes(n))
    keys = torch.empty(2 * n, dtype=torch.int32, device="cuda")
    rows = torch.empty(n, dtype=torch.int32, device="cuda")
    perm = torch.empty(n, dtype=torch.int32, device="cuda")
    tmp = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
    c = fast.c
    assert L.evx_act_row_perm(C.byref(lay.c), obs.data_ptr(), n, int(c.stat_fs), int(c.stat_x0), int(c.stat_nx),
                              keys.data_ptr(), rows.data_ptr(), perm.data_ptr(), tmp.data_ptr(), tmp.numel(), None) == 0
    # too little temp storage is refused before anything is launched
    assert L.evx_act_row_perm(C.byref(lay.c), obs.data_ptr(), n, int(c.stat_fs), int(c.stat_x0), int(c.stat_nx),
                              keys.data_ptr(), rows.data_ptr(), perm.data_ptr(), tmp.data_ptr(), 0, None) != 0
    return perm


@pytest.mark.parametrize("all_table", [True, False])
def test_row_permuted_act_matches(all_table):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qnet import DROPOUT_P, Learner
    E, R = 1024, 16
    n = E * R
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), 2276)
    env = VecEnv(lay, E)
    env.seed([300 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(9)
    for _ in range(60):
        env.step(torch.randint(0, 5, (n,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    torch.cuda.synchronize()
    c = lay.c
    lr = Learner(kind="mlp", precision="f32", seed=3)
    lr.fast.attach_static(c, c.L, c.W, c.t_max, x_range=(max(c.rx_lo, 0), min(c.rx_hi, c.L + 1)))
    obs = env.obs.view(-1, 8).clone()
    if all_table:
        obs[:, 6] = int(c.t_max)
    else:  # every other env at the last fire step: the order must gather the table rows first
        obs.view(E, R, 8)[::2, :, 6] = int(c.t_max)
    perm = _row_perm(lay, obs, n, lr.fast)
    # keys restated: not-on-table bit 20, centre x (W + 2) + y; stable argsort
    o = obs.cpu().numpy()
    fs = np.clip(o[:, 6], 0, c.t_max)
    x0, nx = int(lr.fast.c.stat_x0), int(lr.fast.c.stat_nx)
    tab = (fs == c.t_max) & (o[:, 4] >= x0) & (o[:, 4] < x0 + nx) & (o[:, 5] >= 0) & (o[:, 5] <= c.W + 1)
    key = np.where(tab, 0, 1 << 20) + np.clip(o[:, 4], 0, c.L + 1) * (c.W + 2) + np.clip(o[:, 5], 0, c.W + 1)
    ref = np.argsort(key, kind="stable")
    p = perm.cpu().numpy()
    assert np.array_equal(p, ref)
    assert np.array_equal(np.sort(p), np.arange(n))
    q0 = torch.empty(n, 5, device="cuda")
    a0 = torch.empty(n, dtype=torch.int32, device="cuda")
    q1 = torch.empty(n, 5, device="cuda")
    a1 = torch.empty(n, dtype=torch.int32, device="cuda")
    drop = (11, 5, DROPOUT_P, None, 0)
    lr.fast.act(lay.c, obs.view(-1), n, drop=drop, q=q0, actions=a0, epsilon=0.3, act_seed=7, act_offset=123)
    lr.fast.act(lay.c, obs.view(-1), n, drop=drop, q=q1, actions=a1, epsilon=0.3, act_seed=7, act_offset=123,
                perm=perm, rows_per_env=1)
    torch.cuda.synchronize()
    assert np.array_equal(a1.cpu().numpy(), orc.epsilon_greedy(q1.cpu().numpy(), 0.3, 7, 123))
    if all_table:
        assert torch.equal(q0, q1) and torch.equal(a0, a1)
    else:
        # rows on the table path in both: the unpermuted act's all-table tiles (64 consecutive
        # rows) and the permuted act's all-table tiles (64 consecutive perm entries)
        t0 = np.repeat(tab.reshape(-1, 64).all(1), 64)
        t1 = np.zeros(n, bool)
        t1[p] = np.repeat(tab[p].reshape(-1, 64).all(1), 64)
        both = t0 & t1
        full0 = np.repeat(~tab.reshape(-1, 64).all(1), 64)  # full path in both: tiles not all on the table
        full1 = np.zeros(n, bool)
        full1[p] = np.repeat(~tab[p].reshape(-1, 64).all(1), 64)
        same = both | (full0 & full1)
        assert same.sum() > n // 4
        m = torch.from_numpy(same).cuda()
        assert torch.equal(q0[m], q1[m])
