"""The value-mixing learn step (evacx.qmix, reference runners/train_qmix.py:78-118) on the
device learners vs the reference's formulation in plain PyTorch fp32 autograd (the same
weights, dropout masks and mixer): loss, each agent's clipped gradients and updated
parameters, the mixer's updated parameters. Tolerances as tests/test_qnet_gpu.py's
exact-f32 path."""
import copy

import pytest
import torch
import torch.nn.functional as F

from test_qnet_gpu import make_batch, torch_forward

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("kind", ["mlp", "conv"])
def test_qmix_step_matches_torch_autograd(kind):
    _need_gpu()
    from evacx.qmix import MixingNetwork, QMixLearnStep
    from evacx.qnet import Learner
    torch.manual_seed(0)
    B = 16
    lrs = [Learner(kind=kind, precision="f32", seed=40 + i, lr=1e-3) for i in range(2)]
    mixing = MixingNetwork(2).cuda()
    tmix = MixingNetwork(2).cuda()
    tmix.load_state_dict(mixing.state_dict())
    ref_mix, ref_tmix = copy.deepcopy(mixing), copy.deepcopy(tmix)
    step = QMixLearnStep(lrs, mixing, tmix, torch.optim.Adam(mixing.parameters(), lr=1e-3), gamma=0.99)
    params = [{k: torch.nn.Parameter(v.cpu().clone()) for k, v in lr.online.state_dict().items()} for lr in lrs]
    tgts = [{k: v.cpu().clone() for k, v in lr.target.state_dict().items()} for lr in lrs]
    opts = [torch.optim.Adam(p.values(), lr=1e-3) for p in params]
    batches = [make_batch(B, 70 + i) for i in range(2)]
    xs = [b[0] for b in batches]
    x2s = [b[1] for b in batches]
    acts = [b[2] for b in batches]
    r = batches[0][3].float()
    d = batches[0][4]
    m_on = [b[5] for b in batches]
    m_tg = [b[6] for b in batches]
    loss = step([x.cuda() for x in xs], [a.cuda() for a in acts], r.cuda(), d.cuda(), [x.cuda() for x in x2s],
                masks=[m.cuda() for m in m_on], target_masks=[m.cuda() for m in m_tg])
    # the reference's formulation
    qs = [torch_forward(kind, params[i], xs[i], m_on[i]).gather(1, acts[i].long().unsqueeze(1)).squeeze()
          for i in range(2)]
    with torch.no_grad():
        nq = [torch_forward(kind, tgts[i], x2s[i], m_tg[i]).max(1)[0] for i in range(2)]
        y = r + 0.99 * ref_tmix.cpu()(torch.stack(nq, 1)) * (~d.bool())
    ref_mix_cpu = ref_mix.cpu()
    ref_mix_opt = torch.optim.Adam(ref_mix_cpu.parameters(), lr=1e-3)
    ref_loss = F.mse_loss(ref_mix_cpu(torch.stack(qs, 1)), y)
    ref_mix_opt.zero_grad()
    for o in opts:
        o.zero_grad()
    ref_loss.backward()
    norms = [torch.nn.utils.clip_grad_norm_(p.values(), 1.0) for p in params]
    torch.nn.utils.clip_grad_norm_(ref_mix_cpu.parameters(), 1.0)
    ref_mix_opt.step()
    for o in opts:
        o.step()
    assert abs(loss.item() - ref_loss.item()) <= 2e-4 * abs(ref_loss.item()) + 1e-5
    for i, lr in enumerate(lrs):
        assert abs(lr.norm.item() - norms[i].item()) <= 2e-4 * norms[i].item() + 1e-6
        for k, p in params[i].items():
            torch.testing.assert_close(lr.grads[k].cpu(), p.grad, rtol=2e-3, atol=2e-6)
            diff = (lr.online[k].cpu() - p.detach()).abs()
            assert (diff > 1e-5).float().mean().item() <= 1e-4, (k, diff.max().item())
    for (n1, p1), (n2, p2) in zip(mixing.named_parameters(), ref_mix_cpu.named_parameters()):
        torch.testing.assert_close(p1.grad.cpu(), p2.grad, rtol=2e-3, atol=1e-6)  # clipped mixer grads
        assert (p1.detach().cpu() - p2.detach()).abs().max().item() <= 1e-3  # within one Adam step (lr)
