"""Worker of tests/test_distributed_gpu.py (not a test module): one rank of a world-W
data-parallel VecTrainer run on cuda:0 with the gradient all-reduce hook over gloo.

    python tests/dist_trainer_worker.py RANK WORLD PORT OUTDIR [uniform|prio]

Writes OUTDIR/w{WORLD}_r{RANK}.npz (prio: OUTDIR/prio_w{WORLD}_r{RANK}.npz):
  * the rank's env states after 8 training steps (global env ids rank*E .. rank*E+E-1 of
    64; epsilon 1.0 without decay, so actions depend only on the global agent id and the
    step -- trajectories must not depend on WORLD);
  * the trainer's online parameters (every rank's must be bit-identical);
  * one Learner.learn_obs on this rank's share of a fixed 128-row union batch (explicit
    dropout masks), after the hook averaged the gradients: clipped gradients, parameters.
prio: cfg5's shape -- 32 robots per env, prioritized replay (per-rank sum/min trees over
the rank's own ring, evacx.prio) -- on a 64x64 layout with 16 envs in all; the rank's trees
and max leaf are saved too, and the union-batch learn carries importance weights and
returns |TD error| (the prioritized learn's inputs and outputs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    prio = len(sys.argv) > 5 and sys.argv[5] == "prio"
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from evacx.qnet import Learner
    from evacx.trainer import VecTrainer, make_allreduce_hook
    if prio:
        E_TOT, R, P, Lg = 16, 32, 569, 64
    else:
        E_TOT, R, P, Lg = 64, 4, 150, 32
    E = E_TOT // world
    lay = DeviceLayout(build_tables(synthetic(Lg, Lg, R)), P)
    hook = make_allreduce_hook(dist, world) if dist is not None else None
    tr = VecTrainer(lay, E, env_offset=rank * E, world_envs=E_TOT, batch=64, replay_capacity=4096, epsilon=1.0,
                    epsilon_decay=1.0, grad_hook=hook, learner_seed=0,
                    replay="prioritized" if prio else "uniform")
    for _ in range(8):
        tr.step()
    tr.sync()
    torch.cuda.synchronize()
    sts = tr.env.host_states(range(E))
    res = {k: np.stack([st[k] for st in sts]) for k in ["pos", "flags", "health", "acc", "rmap", "robots", "view",
                                                       "scal", "py_mt", "np_mt"]}
    res["trainer_params"] = tr.learner.online.flat.cpu().numpy()
    res["learn_steps"] = np.int64(tr.learn_steps)
    if prio:
        res["tsum"] = tr.replay.tsum.cpu().numpy()
        res["tmin"] = tr.replay.tmin.cpu().numpy()
        res["max_leaf"] = tr.replay.max_leaf.cpu().numpy()
        res["replay_size"] = np.int64(tr.replay.size)

    # learner: this rank's share of a fixed union batch, gradients averaged by the hook
    NE = 32 if not prio else 4  # the union batch: 128 observations
    venv = VecEnv(lay, NE)
    venv.seed(list(range(500, 500 + NE)))
    venv.reset()
    g = torch.Generator().manual_seed(9)
    for _ in range(3):
        venv.step(torch.randint(0, 5, (NE * R,), generator=g, dtype=torch.int32).cuda())
    obs = venv.obs.view(-1, 8).clone()
    NU = obs.shape[0]
    perm = torch.randperm(NU, generator=g).cuda()
    a = torch.randint(0, 5, (NU,), generator=g, dtype=torch.int32).cuda()
    r = (torch.randn(NU, generator=g) * 20).cuda()
    d = (torch.rand(NU, generator=g) < 0.2).to(torch.uint8).cuda()
    m1 = (torch.rand(NU, 512, generator=g) >= 0.2).to(torch.uint8).cuda()
    m2 = (torch.rand(NU, 512, generator=g) >= 0.2).to(torch.uint8).cuda()
    B = NU // world
    rows = slice(rank * B, (rank + 1) * B)
    lr = Learner(kind="mlp", precision="f32", seed=3, lr=1e-3)
    lr.grad_hook = hook
    w = td = None
    if prio:  # importance weights in, |TD error| out (the prioritized learn)
        w = (0.25 + torch.rand(NU, generator=g)).cuda()[rows].contiguous()
        td = torch.zeros(B, dtype=torch.float32, device="cuda")
    loss = lr.learn_obs(lay.c, obs[rows].contiguous().view(-1), a[rows], r[rows], d[rows],
                        obs[perm][rows].contiguous().view(-1), B, mask_online=m1[rows], mask_target=m2[rows],
                        weights=w, td_abs=td)
    torch.cuda.synchronize()
    if prio:
        res["learn_td"] = td.cpu().numpy()
    res["learn_grads"] = lr.grads.flat.cpu().numpy()
    res["learn_params"] = lr.online.flat.cpu().numpy()
    res["learn_norm"] = np.float64(lr.norm.item())
    res["learn_loss"] = np.float64(loss.item())
    np.savez(os.path.join(out, f"{'prio_' if prio else ''}w{world}_r{rank}.npz"), **res)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
