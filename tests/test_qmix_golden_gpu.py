"""The device QMIX mixer (evx_qmix_loss + the mixer's evx_sumsq_norm / evx_clip_adam, the launches
evacx.qgroup.GroupedQMix makes) against the reference's own MixingNetwork learn steps
(tests/golden/qmix_mixer.npz, runners/train_qmix.py:39-113; see tests/test_qmix_golden_cpu.py).
Q / Qt [2][B][5] are built so that the taken actions' Q are the fixture's chosen Q-values and
each row's max over actions of Qt is the fixture's target max. Checked per step: the loss,
d loss / d Q at the taken actions (zero elsewhere), the raw mixer gradient, the norm, and the
mixer parameters after clip + Adam. Tolerances: f32 reassociation (rtol 1e-4 on the sums over
B = 32 rows and 32 hidden units; parameters within 1e-6 of lr scale)."""
import pytest
import torch

from golden_util import load

pytestmark = pytest.mark.gpu


def test_device_mixer_matches_reference_steps():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ctypes as C
    from evacx.qmlp import mlib
    from evacx.qnet import evx_adam, qcheck, qlib
    fx = load("qmix_mixer")
    names = [str(n) for n in fx["names"]]
    n, A, dev = 2, 5, "cuda"
    flat = torch.cat([torch.from_numpy(fx["init_" + k]).reshape(-1) for k in names]).to(dev)
    nm = int(mlib().evx_qmix_nparams(n))
    assert nm == flat.numel()
    flat_t = flat.clone()
    m, v, grad = torch.zeros_like(flat), torch.zeros_like(flat), torch.zeros_like(flat)
    loss, norm = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
    scratch = torch.zeros(2048, device=dev)
    g = torch.Generator().manual_seed(3)
    for s in range(3):
        p = f"s{s}_"
        q = torch.from_numpy(fx[p + "q"])    # [B][2]
        tq = torch.from_numpy(fx[p + "tq"])  # [B][2]
        B = q.shape[0]
        act = torch.randint(0, A, (n, B), generator=g, dtype=torch.int32)
        Q = torch.randn(n, B, A, generator=g) * 3
        Q.scatter_(2, act.long().unsqueeze(2), q.t().unsqueeze(2))
        Qt = tq.t().unsqueeze(2) - torch.rand(n, B, A, generator=g) * 5 - 0.01  # below the max ...
        Qt.scatter_(2, torch.randint(0, A, (n, B, 1), generator=g), tq.t().unsqueeze(2))  # ... which one action holds
        rew = torch.from_numpy(fx[p + "r"])
        done = torch.from_numpy(fx[p + "d"])
        # raw pointers below: [n][B][A] contiguous (the broadcast above may leave Qt's strides permuted)
        Q, Qt, act, rew, done = [t.contiguous().to(dev) for t in (Q, Qt, act, rew, done)]
        dQ = torch.full((n, B, A), 7.0, device=dev)
        part = torch.empty(int(mlib().evx_qmix_part_floats(B, n)), device=dev)
        zero = torch.ones(64, device=dev)
        rc = mlib().evx_qmix_loss(Q.data_ptr(), Qt.data_ptr(), A, act.data_ptr(), rew.data_ptr(), done.data_ptr(),
                                  0.99, B, n, flat.data_ptr(), flat_t.data_ptr(), dQ.data_ptr(), grad.data_ptr(),
                                  loss.data_ptr(), part.data_ptr(), zero.data_ptr(), zero.numel(), None)
        assert rc == 0
        L = qlib()
        qcheck(L.evx_sumsq_norm(grad.data_ptr(), nm, scratch.data_ptr(), scratch.numel(), norm.data_ptr(), None),
               "sumsq")
        raw = grad.clone()
        h = evx_adam(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=s + 1)
        qcheck(L.evx_clip_adam(flat.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(), nm, norm.data_ptr(), 1.0,
                               C.byref(h), None), "clip_adam")
        torch.cuda.synchronize()
        ref_loss = float(fx[p + "loss"])
        assert abs(loss.item() - ref_loss) <= 1e-4 * abs(ref_loss), (s, loss.item(), ref_loss)
        assert abs(norm.item() - float(fx[p + "norm"])) <= 1e-4 * float(fx[p + "norm"]), s
        assert torch.count_nonzero(zero) == 0
        dref = torch.zeros(n, B, A)
        dref.scatter_(2, act.cpu().long().unsqueeze(2), torch.from_numpy(fx[p + "dq"]).t().unsqueeze(2))
        torch.testing.assert_close(dQ.cpu(), dref, rtol=1e-4, atol=1e-6 * dref.abs().max().item())
        raw_ref = torch.cat([torch.from_numpy(fx[p + "raw_" + k]).reshape(-1) for k in names])
        torch.testing.assert_close(raw.cpu(), raw_ref, rtol=1e-4, atol=1e-5 * raw_ref.abs().max().item())
        pref = torch.cat([torch.from_numpy(fx[p + "param_" + k]).reshape(-1) for k in names])
        assert (flat.cpu() - pref).abs().max().item() <= 1e-6 + 1e-6 * pref.abs().max().item(), s
