"""x3 vs exact-f32 conv learner: the 3 steps of tests/test_qnet_gpu.py::test_learn_steps_match_torch_adam,
per-tensor max gradient error / max |grad| against torch f32, and the count of conv pre-activations
whose sign differs from torch's (relu gate flips)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "dqn-marl_amd"))
import torch, torch.nn.functional as F
from test_qnet_gpu import make_batch, torch_forward
from evacx.qnet import Learner

B = 32
for prec in ("f32", "x3"):
    lr = Learner(kind="conv", precision=prec, seed=5, lr=1e-3)
    sd0 = {k: v.cpu().clone() for k, v in lr.online.state_dict().items()}
    params = {k: torch.nn.Parameter(v.clone()) for k, v in sd0.items()}
    tgt = {k: v.clone() for k, v in sd0.items()}
    opt = torch.optim.Adam(params.values(), lr=1e-3)
    for it in range(3):
        if it > 0:
            lr.online.load_state_dict({k: p.detach() for k, p in params.items()})
            for key, buf in (("exp_avg", lr.m), ("exp_avg_sq", lr.v)):
                buf.copy_(torch.cat([opt.state[p][key].reshape(-1) for p in params.values()]).cuda())
        x, x2, a, r, d, m1, m2 = make_batch(B, 10 + it)
        lr.learn(x.cuda(), a.cuda(), r.float().cuda(), d.cuda(), x2.cuda(), m1.cuda(), m2.cuda())
        # relu flips in the conv stack: pre-activation of torch vs the saved GPU activations
        h = x.permute(0, 3, 1, 2).contiguous()
        flips = []
        for li, c in enumerate(("conv1", "conv2", "conv3")):
            z = F.conv2d(h, params[c + ".weight"].detach(), params[c + ".bias"].detach(), padding=1)
            yg = lr.net.saved["ys"][li].cpu().reshape(B, 11, 11, -1).permute(0, 3, 1, 2)
            flips.append(int(((z > 0) != (yg > 0)).sum()))
            h = F.relu(z)
        q = torch_forward("conv", params, x, m1).gather(1, a.long().unsqueeze(1))
        with torch.no_grad():
            nq = torch_forward("conv", tgt, x2, m2).max(1)[0]
            y = r.float() + 0.99 * nq * (~d.bool())
        opt.zero_grad()
        F.mse_loss(q.squeeze(), y).backward()
        torch.nn.utils.clip_grad_norm_(params.values(), 1.0)
        errs = {k: (lr.grads[k].cpu() - p.grad).abs().max().item() / p.grad.abs().max().item()
                for k, p in params.items()}
        opt.step()
        print(prec, it, "flips", flips, " ".join(f"{k.split('.')[0]}{k[-1]}:{v:.1e}" for k, v in errs.items()))
