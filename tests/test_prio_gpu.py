"""GPU prioritized replay (csrc/prio.hip) against the oracle (oracle/prio_oracle.c).

Trees are compared bit for bit (every internal node is left + right / min of its
children, so they are a pure function of the leaves); leaf priorities (td + eps)^alpha
come from the device pow and the C library pow, compared within 1 ulp, after which the
oracle adopts the GPU's leaves. Sample indices are exact; importance weights within one
float32 ulp (pow again)."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ring(C):
    from evacx.prio import PrioReplay
    rp = PrioReplay(C, "cuda")
    # distinct payloads so gathers can be checked: action = slot, reward = slot / 2
    rp.a.copy_(torch.arange(C, dtype=torch.int32, device="cuda"))
    rp.r.copy_(torch.arange(C, dtype=torch.float32, device="cuda") * 0.5)
    rp.s.view(C, -1)[:, 0] = torch.arange(C, dtype=torch.int32, device="cuda")
    return rp


def _adopt_leaves(o, rp):
    """Leaves within 1 ulp, then the oracle takes the GPU's leaves and rebuilds."""
    C = o.C
    gs, gm = rp.tsum.cpu().numpy(), rp.tmin.cpu().numpy()
    ls, lm = gs[C:], gm[C:]
    fin = np.isfinite(o.mn[C:])
    assert np.all(np.abs(ls - o.sum[C:]) <= np.spacing(np.maximum(np.abs(o.sum[C:]), 1e-300)))
    assert np.array_equal(np.isfinite(lm), fin)
    o.sum[C:] = ls
    o.mn[C:] = lm
    o.set_range(0, 0, 0)  # rebuild only
    assert np.array_equal(gs[1:], o.sum[1:]), "sum tree"
    assert np.array_equal(gm[1:], o.mn[1:]), "min tree"
    o.max_leaf[0] = rp.max_leaf.item()


@pytest.mark.parametrize("C", [1024, 1 << 15, 1 << 20, 1 << 22])  # 2^22: cfg5's ring, a three-pass rebuild
def test_trees_and_sampling_vs_oracle(C):
    _need_gpu()
    rp = _ring(C)
    o = orc.PrioTrees(C)
    rng = np.random.RandomState(C & 0xFFFF)
    from evacx.env import OBS_WORDS
    B = 4096
    out = dict(s=torch.zeros(B * OBS_WORDS, dtype=torch.int32, device="cuda"),
               s2=torch.zeros(B * OBS_WORDS, dtype=torch.int32, device="cuda"),
               a=torch.zeros(B, dtype=torch.int32, device="cuda"), r=torch.zeros(B, device="cuda"),
               done=torch.zeros(B, dtype=torch.uint8, device="cuda"))
    idx = torch.zeros(B, dtype=torch.int64, device="cuda")
    w = torch.zeros(B, device="cuda")
    pos = C - C // 3  # ranges wrap
    for it in range(6):
        n_new = int(rng.randint(1, C // 2))
        n_hide = int(rng.randint(0, C // 4)) if it % 2 else 0
        rp.pos, rp.unexposed = (pos + n_new) % C, n_new
        rp.expose(n_hide=n_hide)
        o.set_range(pos, n_new, n_hide)
        pos = (pos + n_new) % C
        torch.cuda.synchronize()
        assert np.array_equal(rp.tsum.cpu().numpy()[1:], o.sum[1:]), (it, "sum after set_range")
        assert np.array_equal(rp.tmin.cpu().numpy()[1:], o.mn[1:]), (it, "min after set_range")
        assert rp.max_leaf.item() == o.max_leaf[0]
        beta = 0.4 + 0.1 * it
        rp.sample_prio(B, beta, 99, it * B, out, idx, w)
        oi, ow = o.sample(B, beta, 99, it * B)
        gi = idx.cpu().numpy()
        assert np.array_equal(gi, oi), (it, "indices")
        gw = w.cpu().numpy()
        assert np.all(np.abs(gw - ow) <= np.spacing(ow)), (it, "weights")
        assert np.array_equal(out["a"].cpu().numpy(), oi.astype(np.int32))
        assert np.array_equal(out["r"].cpu().numpy(), (oi * 0.5).astype(np.float32))
        assert np.array_equal(out["s"].view(B, -1)[:, 0].cpu().numpy(), oi.astype(np.int32))
        assert np.all(o.sum[C + oi] > 0)  # never an empty or hidden slot
        # priorities of the sampled slots from TD errors, duplicates included
        td = (rng.rand(B) * 3).astype(np.float32)
        td_t = torch.from_numpy(td).cuda()
        rp.update(idx, td_t, B)
        o.update(oi, td, rp.eps, rp.alpha)
        torch.cuda.synchronize()
        _adopt_leaves(o, rp)


def test_trainer_prioritized_strict_and_lagged():
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    lay = DeviceLayout(build_tables(synthetic(64, 64, 8)), 569)
    for lagged in (False, True):
        tr = VecTrainer(lay, 64, batch=256, replay_capacity=1 << 12, lagged_learn=lagged, replay="prioritized")
        for _ in range(30):
            tr.step()
        tr.sync()
        torch.cuda.synchronize()
        assert tr.learn_steps > 0
        assert np.isfinite(tr.last_loss.item())
        C = tr.replay.capacity
        s = tr.replay.tsum.cpu().numpy()
        o = orc.PrioTrees(C)
        o.sum[:] = s
        o.mn[:] = tr.replay.tmin.cpu().numpy()
        o.set_range(0, 0, 0)
        assert np.array_equal(o.sum, s)  # internal nodes consistent with the leaves
        if lagged:  # the slots the next push overwrites are hidden
            hid = (tr.replay.pos - tr.n_agents + np.arange(tr.n_agents)) % C  # push t's slots
            assert np.all(s[C + hid] == 0)
        w = tr.samp["w"].cpu().numpy()
        assert np.all(w > 0) and np.all(w <= 1.0)
