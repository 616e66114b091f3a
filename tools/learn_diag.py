"""Diagnostic: the x3 learn chain's gradient error vs batch size (tests/test_bench_scale_gpu.py).

For each B: one learn_obs step from compact observations of a 128x128 R16 env, against an
f64 torch autograd reference (and the f32 torch restatement, to see the reference's own
error). Prints, per gradient tensor, max |err| / max |ref| and the count of elements that fail
the tests' criterion (rtol 2e-3, atol 1e-5 max|ref|); for fc1.weight also the centre column
(365) and the channels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def tq(sd, X, mask):
    h = F.relu(F.linear(X, sd["fc1.weight"], sd["fc1.bias"]))
    h = h * mask.to(h.dtype) / 0.8
    h = F.relu(F.linear(h, sd["fc2.weight"], sd["fc2.bias"]))
    return F.linear(h, sd["fc3.weight"], sd["fc3.bias"])


def ref_grads(sd0, X, X2, a, r, d, m1, m2, dtype):
    p = {k: torch.nn.Parameter(v.to(dtype).clone()) for k, v in sd0.items()}
    t = {k: v.to(dtype) for k, v in sd0.items()}
    q = tq(p, X.to(dtype), m1).gather(1, a.long().unsqueeze(1))
    with torch.no_grad():
        y = r.to(dtype) + 0.99 * tq(t, X2.to(dtype), m2).max(1)[0] * (~d.bool())
    loss = F.mse_loss(q.squeeze(), y)
    loss.backward()
    return loss.item(), {k: v.grad for k, v in p.items()}


def main():
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qmlp import HID, K1
    from evacx.qnet import Learner
    R, P = 16, 2276
    Bs = [int(b) for b in (sys.argv[1:] or ["512", "2048", "4096", "8192", "32768"])]
    Emax = 2 * max(Bs) // R
    lay = DeviceLayout(build_tables(synthetic(128, 128, R)), P)
    env = VecEnv(lay, Emax)
    env.seed([500 + i for i in range(Emax)])
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(40):
        env.step(torch.randint(0, 5, (Emax * R,), device="cuda", dtype=torch.int32, generator=g), auto_reset=True)
    obs = env.obs.view(-1, 8)
    for B in Bs:
        lr = Learner(kind="mlp", precision="f32", seed=41, lr=1e-3)
        sd0 = {k: v.clone() for k, v in lr.online.state_dict().items()}
        gh = torch.Generator().manual_seed(B)
        perm = torch.randperm(Emax * R, generator=gh)
        s_obs = obs[perm[:B].cuda()].contiguous().view(-1)
        s2_obs = obs[perm[B:2 * B].cuda()].contiguous().view(-1)
        a = torch.randint(0, 5, (B,), generator=gh, dtype=torch.int32).cuda()
        r = (torch.randn(B, generator=gh) * 30).cuda()
        d = (torch.rand(B, generator=gh) < 0.05).to(torch.uint8).cuda()
        m1 = (torch.rand(B, HID, generator=gh) >= 0.2).to(torch.uint8).cuda()
        m2 = (torch.rand(B, HID, generator=gh) >= 0.2).to(torch.uint8).cuda()
        lr.max_norm = 0.0  # raw gradients (no clip) for the comparison
        loss = lr.learn_obs(lay.c, s_obs, a, r, d, s2_obs, B, mask_online=m1, mask_target=m2, update=False)
        torch.cuda.synchronize()
        X = env.expand_obs(torch.float32, s_obs).reshape(B, K1)
        X2 = env.expand_obs(torch.float32, s2_obs).reshape(B, K1)
        l64, g64 = ref_grads(sd0, X, X2, a, r, d, m1, m2, torch.float64)
        l32, g32 = ref_grads(sd0, X, X2, a, r, d, m1, m2, torch.float32)
        print(f"B={B}: loss dev {loss.item():.8g} f32 {l32:.8g} f64 {l64:.8g}")
        for k in g64:
            ref = g64[k]
            sc = ref.abs().max().item()
            for tag, got in (("dev", lr.grads[k].double()), ("t32", g32[k].double())):
                err = (got - ref).abs()
                bad = (err > 2e-3 * ref.abs() + 1e-5 * sc).sum().item()
                print(f"  {k:11s} {tag} max|err|/max|ref| {err.max().item() / sc:.3e}  fails {bad}/{ref.numel()}"
                      f"  at {tuple(int(i) for i in torch.nonzero(err == err.max())[0].tolist())}")
            if k == "fc1.weight":
                got = lr.grads[k].double()
                err = (got - ref).abs()
                print(f"    centre col: max|err| {err[:, 365].max().item():.3e} max|ref| {ref[:, 365].abs().max().item():.3e}"
                      f"; t32 {(g32[k].double() - ref)[:, 365].abs().max().item():.3e}")
                for ch in range(6):
                    e = err.view(HID, 121, 6)[:, :, ch]
                    rr = ref.view(HID, 121, 6)[:, :, ch]
                    print(f"    ch{ch}: max|err| {e.max().item():.3e} max|ref| {rr.abs().max().item():.3e}")
        gb = lr.grads["fc1.bias"].double()
        print(f"    db1 vs dW1[:,365] (dev) max diff {(gb - lr.grads['fc1.weight'][:, 365].double()).abs().max().item():.3e}")


if __name__ == "__main__":
    main()
