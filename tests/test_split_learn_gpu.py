"""The split learn step (evacx.trainer.VecTrainer, strict schedule) against the one-part learn.

VecTrainer learns batch t in two row parts: the rows drawn from the ring's slots before push t
(forward + backward on the learn stream beside act t and env.step t) and the rows drawn from
push t's slots (after the push), then clip + Adam. Learner.learn_obs(part=(B, first, last))
carries it: loss and dQ are means over the whole B (evx_td_loss_part), the backward of the later
part accumulates into the gradients the first part left, and only the last part leaves the
clip norm's partials. DQNAgent.learn (agents/dqn_agent.py:126-168) is one step over the whole
batch; here the same batch, dropout masks and parameters go through both and must agree up to
f32 summation order: loss and norm rtol 1e-5, clipped gradients rtol 1e-4 with atol 1e-6 of
the tensor's max, parameters within 1e-6 except where a near-zero gradient flips Adam's first
step (the criterion of tests/test_distributed_gpu.py). Part sizes are odd and uneven, the
fresh part about one sixteenth of B as in the bench (E*R / replay capacity)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,k", [(4096, 257), (32768, 2047), (512, 512)])
def test_split_learn_matches_one_part(B, k):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qmlp import HID
    from evacx.qnet import Learner
    R, P = 16, 2276
    E = 2 * B // R
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), P)
    env = VecEnv(lay, E)
    env.seed([700 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(30):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    torch.cuda.synchronize()
    la = Learner(kind="mlp", precision="f32", seed=5, lr=1e-3)
    lb = Learner(kind="mlp", precision="f32", seed=5, lr=1e-3)
    assert lb.fused_opt and torch.equal(la.online.flat, lb.online.flat)
    gh = torch.Generator().manual_seed(B + k)
    obs = env.obs.view(-1, 8)
    n1 = B - k
    for it in range(2):
        if it:  # the second step from identical state again (isolates one step's arithmetic)
            for dst, src in ((lb.online.flat, la.online.flat), (lb.m, la.m), (lb.v, la.v)):
                dst.copy_(src)
            lb.fast.repack()
        perm = torch.randperm(E * R, generator=gh)
        s_obs = obs[perm[:B].cuda()].contiguous().view(-1)
        s2_obs = obs[perm[B:2 * B].cuda()].contiguous().view(-1)
        a = torch.randint(0, 5, (B,), generator=gh, dtype=torch.int32).cuda()
        r = (torch.randn(B, generator=gh) * 30).cuda()
        d = (torch.rand(B, generator=gh) < 0.05).to(torch.uint8).cuda()
        m1 = (torch.rand(B, HID, generator=gh) >= 0.2).to(torch.uint8).cuda()
        m2 = (torch.rand(B, HID, generator=gh) >= 0.2).to(torch.uint8).cuda()
        loss_a = la.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B, mask_online=m1, mask_target=m2).item()
        if n1:
            lb.learn_obs(lay.c, s_obs, a, r, d, s2_obs, n1, update=False, part=(B, True, False),
                         mask_online=m1[:n1].contiguous(), mask_target=m2[:n1].contiguous())
        lb.learn_obs(lay.c, s_obs[n1 * 8:], a[n1:], r[n1:], d[n1:], s2_obs[n1 * 8:], k, update=False,
                     part=(B, n1 == 0, True), mask_online=m1[n1:].contiguous(), mask_target=m2[n1:].contiguous())
        lb.step_optimizer()
        torch.cuda.synchronize()
        loss_b = lb.loss.item()
        assert abs(loss_a - loss_b) <= 1e-5 * abs(loss_a), (it, loss_a, loss_b)
        assert abs(la.norm.item() - lb.norm.item()) <= 1e-5 * la.norm.item(), (it, la.norm.item(), lb.norm.item())
        for name in la.online.state_dict():
            ga, gb = la.grads[name], lb.grads[name]
            torch.testing.assert_close(gb, ga, rtol=1e-4, atol=1e-6 * ga.abs().max().item() + 1e-12,
                                       msg=lambda m: f"B={B} k={k} step {it} grad {name}: {m}")
        diff = (la.online.flat - lb.online.flat).abs()
        assert (diff > 1e-6).float().mean().item() <= 1e-3 and diff.max().item() <= 2.1e-3, (it, diff.max().item())


def test_split_learn_part_arguments():
    """learn_obs refuses a part larger than its batch and weights in parts; evx_td_loss_part
    refuses B_norm < B and a later part that would clear the gradients."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from evacx.qnet import Learner, qlib
    lr = Learner(kind="mlp", precision="f32", seed=1)
    z = torch.zeros(64 * 8, dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        lr.learn_obs(None, z, None, None, None, z, 64, part=(32, True, True))
    with pytest.raises(ValueError):
        lr.learn_obs(None, z, None, None, None, z, 32, part=(64, True, True), weights=torch.ones(32, device="cuda"))
    q = torch.zeros(64, 5, device="cuda")
    L = qlib()
    one = torch.zeros(1, device="cuda")
    assert L.evx_td_loss_part(q.data_ptr(), q.data_ptr(), 5, None, None, None, 0.99, 64, 32, 0, q.data_ptr(),
                              one.data_ptr(), None, 0, None) != 0
    assert L.evx_td_loss_part(q.data_ptr(), q.data_ptr(), 5, None, None, None, 0.99, 64, 64, 1, q.data_ptr(),
                              one.data_ptr(), one.data_ptr(), 1, None) != 0
    assert np.isfinite(one.item())
