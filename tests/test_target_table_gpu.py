"""The learner's target forward from the target net's act table (evacx.trainer attaches a table to
both nets; csrc/qmlp.hip evx_qmlp_forward2: at B >= 32768 the target Q runs through the fused act
kernel, whose 64-row tiles whose rows all sit past the fire's last step start fc1 from the table
of static features x W1 instead of the full 640-deep contraction).

DQNAgent.learn's target (agents/dqn_agent.py:143-151) is max_a Q_tgt(s') with dropout; the table
path changes only the f32 summation order of fc1's static part. Same batch, masks and parameters
through a learner whose target net has the table and one without: loss and clip norm rtol 1e-5,
clipped gradients rtol 1e-4 (atol 1e-6 of the tensor's max), parameters within 1e-6 except where
a near-zero gradient flips Adam's first step (tests/test_distributed_gpu.py's criterion). Three
quarters of the s' rows are moved to the last fire step (whole tiles take the table path), the rest
stay at their own (full path), and the table is checked to follow a target sync."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_target_table_matches_full_path():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qmlp import HID
    from evacx.qnet import Learner
    B, R, P = 32768, 16, 2276
    E = 2 * B // R
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), P)
    env = VecEnv(lay, E)
    env.seed([900 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(30):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    torch.cuda.synchronize()
    c = lay.c
    la = Learner(kind="mlp", precision="f32", seed=7, lr=1e-3)
    lb = Learner(kind="mlp", precision="f32", seed=7, lr=1e-3)
    xr = (max(c.rx_lo, 0), min(c.rx_hi, c.L + 1))
    lb.fast_t.attach_static(c, c.L, c.W, c.t_max, x_range=xr)
    gh = torch.Generator().manual_seed(17)
    obs = env.obs.view(-1, 8)
    for it in range(3):
        for dst, src in ((lb.online.flat, la.online.flat), (lb.m, la.m), (lb.v, la.v)):
            dst.copy_(src)
        lb.fast.repack()
        if it == 2:  # a target sync: the table follows the new target weights
            for l in (la, lb):
                l.sync_target()
        perm = torch.randperm(E * R, generator=gh)
        s_obs = obs[perm[:B].cuda()].contiguous()
        s2_obs = obs[perm[B:2 * B].cuda()].contiguous()
        s2_obs[:3 * B // 4, 6] = int(c.t_max)
        s_obs, s2_obs = s_obs.view(-1), s2_obs.view(-1)
        a = torch.randint(0, 5, (B,), generator=gh, dtype=torch.int32).cuda()
        r = (torch.randn(B, generator=gh) * 30).cuda()
        d = (torch.rand(B, generator=gh) < 0.05).to(torch.uint8).cuda()
        m1 = (torch.rand(B, HID, generator=gh) >= 0.2).to(torch.uint8).cuda()
        m2 = (torch.rand(B, HID, generator=gh) >= 0.2).to(torch.uint8).cuda()
        loss_a = la.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B, mask_online=m1, mask_target=m2).item()
        loss_b = lb.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B, mask_online=m1, mask_target=m2).item()
        torch.cuda.synchronize()
        assert abs(loss_a - loss_b) <= 1e-5 * abs(loss_a), (it, loss_a, loss_b)
        assert abs(la.norm.item() - lb.norm.item()) <= 1e-5 * la.norm.item(), (it, la.norm.item(), lb.norm.item())
        for name in la.online.state_dict():
            ga, gb = la.grads[name], lb.grads[name]
            torch.testing.assert_close(gb, ga, rtol=1e-4, atol=1e-6 * ga.abs().max().item() + 1e-12,
                                       msg=lambda m: f"step {it} grad {name}: {m}")
        diff = (la.online.flat - lb.online.flat).abs()
        assert (diff > 1e-6).float().mean().item() <= 1e-3 and diff.max().item() <= 2.1e-3, (it, diff.max().item())


def test_online_table_matches_full_path():
    """The online forward through the act kernel's table path (evx_qmlp_forward2 when the online
    net has its act table, as VecTrainer attaches it: x_expand_kernel + qact3h_kernel SAVE) vs
    qfc1 + qfc23, from the same parameters: X bit-identical (the same compact input the backward's
    dW1 reads); H1 (hi + lo) and Q within 2e-5 of their scale; the loss rtol 1e-4. Gradients are
    not compared here: a pre-activation within an x3 rounding of 0 may take the other ReLU branch
    on either path, moving its row's whole contribution -- test_bench_scale_gpu.py::
    test_x3_learn_at_bench_batch[table] checks this path's gradients and Adam update against torch
    autograd through the device's own branch pattern. Three quarters of the s rows at the last fire
    step (table tiles), the rest at their own (full-path tiles of the same kernel)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qmlp import HID
    from evacx.qnet import Learner
    B, R, P = 32768, 16, 2276
    E = 2 * B // R
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), P)
    env = VecEnv(lay, E)
    env.seed([700 + i for i in range(E)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(30):
        env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    torch.cuda.synchronize()
    c = lay.c
    la = Learner(kind="mlp", precision="f32", seed=7, lr=1e-3)
    lb = Learner(kind="mlp", precision="f32", seed=7, lr=1e-3)
    xr = (max(c.rx_lo, 0), min(c.rx_hi, c.L + 1))
    lb.fast.attach_static(c, c.L, c.W, c.t_max, x_range=xr)
    gh = torch.Generator().manual_seed(29)
    obs = env.obs.view(-1, 8)
    dev = torch.device("cuda")
    for it in range(3):
        for dst, src in ((lb.online.flat, la.online.flat), (lb.m, la.m), (lb.v, la.v)):
            dst.copy_(src)
        lb.fast.repack()  # (also rebuilds lb's online table from the copied weights)
        perm = torch.randperm(E * R, generator=gh)
        s_obs = obs[perm[:B].cuda()].contiguous()
        s2_obs = obs[perm[B:2 * B].cuda()].contiguous()
        s_obs[:3 * B // 4, 6] = int(c.t_max)
        s_obs, s2_obs = s_obs.view(-1), s2_obs.view(-1)
        a = torch.randint(0, 5, (B,), generator=gh, dtype=torch.int32).cuda()
        r = (torch.randn(B, generator=gh) * 30).cuda()
        d = (torch.rand(B, generator=gh) < 0.05).to(torch.uint8).cuda()
        loss_a = la.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B).item()
        loss_b = lb.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B).item()
        torch.cuda.synchronize()
        xa = la.net.ws.get("fx", (B * la.fast.kx,), torch.int16, dev)
        xb = lb.net.ws.get("fx", (B * lb.fast.kx,), torch.int16, dev)
        assert torch.equal(xa, xb), it
        qa = la.net.ws.get("fq", (B * la.actions,), torch.float32, dev)
        qb = lb.net.ws.get("fq", (B * lb.actions,), torch.float32, dev)
        assert (qa - qb).abs().max().item() <= 2e-5 * qa.abs().max().item(), it
        assert abs(loss_a - loss_b) <= 1e-4 * abs(loss_a), (it, loss_a, loss_b)
        ha = la.net.ws.get("fh1", (2 * B * HID,), torch.int16, dev).view(torch.bfloat16).view(2, B, HID).float().sum(0)
        hb = lb.net.ws.get("fh1", (2 * B * HID,), torch.int16, dev).view(torch.bfloat16).view(2, B, HID).float().sum(0)
        assert (ha - hb).abs().max().item() <= 2e-5 * ha.abs().max().item(), it
