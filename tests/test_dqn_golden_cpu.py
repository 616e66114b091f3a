"""The learner's torch restatement pinned to the reference's own DQNNetwork / DQNAgent.learn.

tests/golden/dqn_forward.npz and dqn_learn.npz were written by tools/capture_golden.py
(dqn_fixtures) from the reference itself (agents/dqn_agent.py:15-168): Q-values of the
full-size conv DQNNetwork and of the MLP variant for closed-form weights
(golden_util.closed_form_params) on observations made by the reference's
EvacuationEnv._get_state, and three DQNAgent.learn steps of each (batch indices from
random.sample, dropout masks from hooks on the Dropout modules, loss, total norm,
pre-clip gradients, parameters and Adam moments after every step).

These CPU tests replay the same arithmetic with the plain-torch restatement the GPU
tests use as their fp32 reference (tests/test_qnet_gpu.py torch_forward + the learn
loop) and require it to reproduce the reference's numbers -- so the GPU learner's
fp32 reference is itself pinned to the reference. Same library (torch CPU), same
operations: agreement within a few f32 ulps (rtol 1e-5, atol 2e-5 of the tensor's scale:
torch's reduction order follows its thread count)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_util import closed_form_params, conv_shapes, load, mlp_shapes, select_positions


def torch_forward(kind, sd, x, mask):
    """agents/dqn_agent.py:35-61 with an injected dropout keep-mask (scale 1/0.8)."""
    B = x.shape[0]
    if kind.startswith("conv"):
        h = x.permute(0, 3, 1, 2).contiguous()
        h = F.relu(F.conv2d(h, sd["conv1.weight"], sd["conv1.bias"], padding=1))
        h = F.relu(F.conv2d(h, sd["conv2.weight"], sd["conv2.bias"], padding=1))
        h = F.relu(F.conv2d(h, sd["conv3.weight"], sd["conv3.bias"], padding=1))
        h = h.reshape(B, -1)
    else:
        h = x.reshape(B, -1)
    h = F.relu(F.linear(h, sd["fc1.weight"], sd["fc1.bias"]))
    if mask is not None:
        h = h * mask.float() / 0.8
    h = F.relu(F.linear(h, sd["fc2.weight"], sd["fc2.bias"]))
    return F.linear(h, sd["fc3.weight"], sd["fc3.bias"])


def shapes_of(kind):
    return conv_shapes(hidden=32) if kind == "conv32" else mlp_shapes()


def test_forward_fixtures_reproduced_by_torch_restatement():
    torch.set_num_threads(4)
    fw = load("dqn_forward")
    lo = load("dqn_learn")
    x = torch.from_numpy(lo["obs"][:16])
    for kind, shapes in [("conv", conv_shapes()), ("mlp", mlp_shapes())]:
        sd = {k: torch.from_numpy(v) for k, v in closed_form_params(shapes, salt=1).items()}
        with torch.no_grad():
            q = torch_forward(kind, sd, x, None)
            torch.testing.assert_close(q, torch.from_numpy(fw[f"{kind}_q_eval"]), rtol=1e-5, atol=1e-6)
            m = torch.from_numpy(fw[f"{kind}_mask_train"])
            q = torch_forward(kind, sd, x, m)
            torch.testing.assert_close(q, torch.from_numpy(fw[f"{kind}_q_train"]), rtol=1e-5, atol=1e-6)
        assert 0.3 < m.float().mean().item() < 0.8  # 0.8 keep x ~half the ReLU outputs positive


@pytest.mark.parametrize("kind", ["conv32", "mlp"])
def test_learn_fixtures_reproduced_by_torch_restatement(kind):
    """DQNAgent.learn (agents/dqn_agent.py:126-168): Q(s).gather(a), r + 0.99 max Q_tgt(s') ~done,
    MSE, backward, clip_grad_norm_(1.0), Adam(lr 1e-4) -- three steps from the same memory."""
    torch.set_num_threads(4)
    lo = load("dqn_learn")
    obs = torch.from_numpy(lo["obs"])
    names = list(shapes_of(kind).keys())
    p0 = closed_form_params(shapes_of(kind), salt=2)
    params = {k: torch.nn.Parameter(torch.from_numpy(v.copy())) for k, v in p0.items()}
    tgt = {k: torch.from_numpy(v.copy()) for k, v in p0.items()}
    opt = torch.optim.Adam(params.values(), lr=1e-4)
    ms, ms2 = lo[f"{kind}_mem_s"], lo[f"{kind}_mem_s2"]
    ma, mr, md = lo[f"{kind}_mem_a"], lo[f"{kind}_mem_r"], lo[f"{kind}_mem_done"]
    for step in range(3):
        idx = lo[f"{kind}_s{step}_idx"]
        s, s2 = obs[ms[idx]], obs[ms2[idx]]
        a = torch.from_numpy(ma[idx].astype(np.int64))
        r = torch.tensor([float(v) for v in mr[idx]], dtype=torch.float32)
        d = torch.from_numpy(md[idx].astype(bool))
        m1 = torch.from_numpy(lo[f"{kind}_s{step}_mask_online"])
        m2 = torch.from_numpy(lo[f"{kind}_s{step}_mask_target"])
        q = torch_forward(kind, params, s, m1).gather(1, a.unsqueeze(1))
        with torch.no_grad():
            y = r + 0.99 * torch_forward(kind, tgt, s2, m2).max(1)[0] * ~d
        loss = F.mse_loss(q.squeeze(), y)
        opt.zero_grad()
        loss.backward()
        pre = {k: p.grad.detach().clone() for k, p in params.items()}
        norm = torch.nn.utils.clip_grad_norm_(params.values(), 1.0)
        opt.step()
        assert abs(loss.item() - lo[f"{kind}_s{step}_loss"]) <= 1e-5 * abs(lo[f"{kind}_s{step}_loss"])
        assert abs(norm.item() - lo[f"{kind}_s{step}_norm"]) <= 1e-5 * lo[f"{kind}_s{step}_norm"]
        for t, k in enumerate(names):
            sel = select_positions(pre[k].numel(), t)
            for tag, val in [("grad", pre[k]), ("param", params[k].detach()), ("m", opt.state[params[k]]["exp_avg"]),
                             ("v", opt.state[params[k]]["exp_avg_sq"])]:
                ref = lo[f"{kind}_s{step}_{tag}_{k}"]
                got = val.reshape(-1).numpy()[sel]
                # summation order inside torch's conv / GEMM depends on the thread count: scale-relative atol
                np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-5 * float(np.abs(ref).max()) + 1e-30,
                                           err_msg=f"{kind} step {step} {tag} {k}")
                ss = float(np.sum(val.reshape(-1).numpy().astype(np.float64) ** 2))
                assert abs(ss - lo[f"{kind}_s{step}_{tag}_{k}__ss"]) <= 1e-5 * lo[f"{kind}_s{step}_{tag}_{k}__ss"] + 1e-30


def test_closed_form_params_deterministic():
    a = closed_form_params(mlp_shapes(), salt=2)
    b = closed_form_params(mlp_shapes(), salt=2)
    for k in a:
        assert np.array_equal(a[k], b[k])
        bound = 1.0 / np.sqrt(726 if k.startswith("fc1") else 512 if k.startswith("fc2") else 256)
        assert np.abs(a[k]).max() <= bound
    assert not np.array_equal(a["fc1.weight"], closed_form_params(mlp_shapes(), salt=1)["fc1.weight"])


def test_flat_params_init_follows_the_global_torch_stream():
    """FlatParams.init_from_global_torch draws the reference DQNNetwork's initial weights
    (nn.Conv2d / nn.Linear reset_parameters in module order, agents/dqn_agent.py:22-31) from
    torch's global generator: same values and the same generator position afterwards."""
    import torch
    import torch.nn as nn

    from collections import OrderedDict

    from evacx.qnet import FlatParams, layer_specs, param_shapes

    def reference_like(h):
        return nn.ModuleDict(OrderedDict([
            ("conv1", nn.Conv2d(6, 32, 3, padding=1)), ("conv2", nn.Conv2d(32, 64, 3, padding=1)),
            ("conv3", nn.Conv2d(64, 128, 3, padding=1)), ("fc1", nn.Linear(11 * 11 * 128, h)),
            ("fc2", nn.Linear(h, h // 2)), ("fc3", nn.Linear(h // 2, 5))]))

    for h in (512, 32):
        torch.manual_seed(77)
        ref = reference_like(h).state_dict()
        after_ref = torch.rand(4)
        torch.manual_seed(77)
        fp = FlatParams(param_shapes(layer_specs("conv", h, 5)), "cpu")
        fp.init_from_global_torch()
        after = torch.rand(4)
        assert list(fp.views) == list(ref)
        for k, v in ref.items():
            assert torch.equal(fp[k], v), (h, k)
        assert torch.equal(after, after_ref)
