"""The device learner against the reference's own DQNNetwork / DQNAgent.learn outputs.

Fixtures (tools/capture_golden.py dqn_fixtures, made by importing the reference): closed-
form weights (golden_util.closed_form_params), observations from the reference's
EvacuationEnv._get_state on the cfg1 layout (with their compact evx_obs forms), Q-values
of the full-size conv DQNNetwork and of the MLP variant, and three DQNAgent.learn steps
(agents/dqn_agent.py:126-168) with the reference's sampled batches and captured dropout
masks. Checked here:
  * evx_obs_expand of the compact forms == the reference's observation tensors (exact);
  * Q-values: the exact-f32 evx_gemm path (conv and MLP) and the fused x3 MLP path,
    rtol 2e-4 / atol 2e-5;
  * learn: loss and total norm rtol 2e-4, clipped gradients rtol 2e-3 (atol 1e-5 of the
    tensor's scale), Adam moments m rtol 2e-3 and v rtol 4e-3 at the stored positions,
    parameters within 2e-7 absolute (lr 1e-4 steps) -- dense f32 path for conv32 and
    MLP, fused x3 path (learn_obs, compact observations) for the MLP."""
import numpy as np
import pytest
import torch

from golden_util import closed_form_params, conv_shapes, load, mlp_shapes, select_positions

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _cfg1():
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, reference_single
    lay = DeviceLayout(build_tables(reference_single()), 150)
    return lay, VecEnv(lay, 1)


def _learner(kind, salt):
    from evacx.qnet import Learner
    hidden = 32 if kind == "conv32" else 512
    lr = Learner(kind="conv" if kind.startswith("conv") else "mlp", precision="f32", hidden=hidden, lr=1e-4, seed=0)
    shapes = conv_shapes(hidden=hidden) if kind.startswith("conv") else mlp_shapes()
    p = closed_form_params(shapes, salt=salt)
    lr.online.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    lr.target.flat.copy_(lr.online.flat)
    if lr.fast is not None:
        lr.fast.repack()
        lr.fast_t.repack()
    return lr, list(shapes.keys())


def test_compact_observations_expand_to_the_reference_tensors():
    _need_gpu()
    lo = load("dqn_learn")
    lay, env = _cfg1()
    comp = torch.from_numpy(lo["obs_compact"]).cuda().view(-1)
    x = env.expand_obs(torch.float64, comp).view(-1, 11, 11, 6).cpu().numpy()
    assert np.array_equal(x.astype(np.float32), lo["obs"])


@pytest.mark.parametrize("kind", ["conv", "mlp"])
def test_forward_matches_reference(kind):
    _need_gpu()
    fw, lo = load("dqn_forward"), load("dqn_learn")
    lr, _ = _learner(kind, salt=1)
    x = torch.from_numpy(lo["obs"][:16]).cuda()
    mask = torch.from_numpy(fw[f"{kind}_mask_train"]).cuda()
    for tag, m in [("eval", None), ("train", mask)]:
        ref = torch.from_numpy(fw[f"{kind}_q_{tag}"])
        q = lr.net.forward(x, m, save=False).cpu()  # evx_gemm, exact f32 MFMA
        torch.testing.assert_close(q, ref, rtol=2e-4, atol=2e-5)
        if kind == "mlp":  # fused x3 path from the compact observations
            from evacx.qmlp import HID
            lay, _ = _cfg1()
            comp = torch.from_numpy(lo["obs_compact"][:16]).cuda().view(-1)
            h1 = torch.empty(2 * 16 * HID, dtype=torch.int16, device="cuda")
            qf = torch.empty(16, 5, device="cuda")
            drop = (0, 0, 0.2, mask) if m is not None else None
            lr.fast.forward(lay.c, comp, 16, h1, drop=drop, q=qf)
            torch.cuda.synchronize()
            torch.testing.assert_close(qf.cpu(), ref, rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("kind,path", [("conv32", "dense"), ("mlp", "dense"), ("mlp", "fused")])
def test_learn_matches_reference(kind, path):
    _need_gpu()
    lo = load("dqn_learn")
    lr, names = _learner(kind, salt=2)
    obs = torch.from_numpy(lo["obs"]).cuda()
    comp = torch.from_numpy(lo["obs_compact"]).cuda()
    lay, _ = _cfg1()
    ms, ms2 = lo[f"{kind}_mem_s"], lo[f"{kind}_mem_s2"]
    ma, mr, md = lo[f"{kind}_mem_a"], lo[f"{kind}_mem_r"], lo[f"{kind}_mem_done"]
    for step in range(3):
        idx = lo[f"{kind}_s{step}_idx"]
        a = torch.from_numpy(ma[idx].astype(np.int32)).cuda()
        r = torch.tensor([float(v) for v in mr[idx]], dtype=torch.float32).cuda()
        d = torch.from_numpy(md[idx].astype(np.uint8)).cuda()
        m1 = torch.from_numpy(lo[f"{kind}_s{step}_mask_online"]).cuda()
        m2 = torch.from_numpy(lo[f"{kind}_s{step}_mask_target"]).cuda()
        si, s2i = torch.from_numpy(ms[idx]).cuda(), torch.from_numpy(ms2[idx]).cuda()
        if path == "dense":
            loss = lr.learn(obs[si], a, r, d, obs[s2i], mask_online=m1, mask_target=m2)
        else:
            loss = lr.learn_obs(lay.c, comp[si].contiguous().view(-1), a, r, d, comp[s2i].contiguous().view(-1),
                                len(idx), mask_online=m1, mask_target=m2)
        torch.cuda.synchronize()
        rl, rn = float(lo[f"{kind}_s{step}_loss"]), float(lo[f"{kind}_s{step}_norm"])
        assert abs(loss.item() - rl) <= 2e-4 * abs(rl), (step, loss.item(), rl)
        assert abs(lr.norm.item() - rn) <= 2e-4 * rn, (step, lr.norm.item(), rn)
        coef = min(1.0, 1.0 / (rn + 1e-6))
        for t, k in enumerate(names):
            n = lr.grads[k].numel()
            sel = torch.from_numpy(select_positions(n, t)).cuda()
            checks = [("grad", lr.grads[k], 2e-3, coef), ("m", lr.m_view(k), 2e-3, 1.0),
                      ("v", lr.v_view(k), 4e-3, 1.0)]
            for tag, val, rtol, scale in checks:
                ref = torch.from_numpy(lo[f"{kind}_s{step}_{tag}_{k}"]).cuda() * scale
                got = val.reshape(-1)[sel]
                torch.testing.assert_close(got, ref, rtol=rtol, atol=1e-5 * ref.abs().max().item() + 1e-30,
                                           msg=lambda m: f"{kind}/{path} step {step} {tag} {k}: {m}")
            ref = torch.from_numpy(lo[f"{kind}_s{step}_param_{k}"]).cuda()
            diff = (lr.online[k].reshape(-1)[sel] - ref).abs().max().item()
            assert diff <= 2e-7 + 1e-6 * ref.abs().max().item(), (kind, path, step, k, diff)
