#!/usr/bin/env python3
"""Benchmark of the evacuation RL hot path on MI355X.

Workload (BASELINE.json metric; configs[2], per-GPU share): synthetic 128x128
layout, 2276 people and 16 robots per env, 4096 envs per GPU (weak scaling;
env ids global, seeds 1234 + global env id), uniform-init MLP Q-net (bf16 MFMA),
batch 4096, replay 2^20 transitions per GPU, gradient all-reduce over RCCL when
world > 1. One timed "step" = one full vectorised training step:
act (Q forward for E*R robots + epsilon-greedy) -> env.step (all E envs, finished
envs auto-reset inside the launch) -> replay push (E*R transitions) -> one learn
step (sample, online+target forward, TD loss, backward, [all-reduce], clip+Adam).
Default schedule "lagged": learn t samples the ring as it stood before push t and
runs on its own stream concurrently with env.step t (the next act waits for it);
"strict" keeps the reference's act -> step -> remember -> learn order, and its rate
on the same state is reported beside the value (strict_schedule_steps_per_s).
Warmup staggers env ages over one episode length (--stagger), so the timed steps
see the stationary mix of episode phases a long training run sees.

value = env-steps/s of the whole job (E * n_gpus * steps / time); the JSON line
also carries agent-transitions/s (x R), the env-only rate, the roofline of the
dominant kernel (env_step_kernel, HBM-bound) and the CPU oracle baseline.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env steps/sec + agent-transitions/sec (whole node), 128x128 grid, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (spec)
EV_EVERY = 5               # timed steps between two HIP-event-bracketed env.step launches


def bytes_per_env_step(P, R, G):
    """Algorithmic HBM bytes of one env-step of env_step_kernel:
    people r+w (pk 4 + health 8 + acc 8) x2, rmap bitmap r+w, two MT19937 states r+w,
    per robot action 4 + position r/w 8 + compact obs 32, per-env scalars 48.
    Shared read-only tables (floor, danger, valid bits) are L2/MALL-resident and excluded."""
    RW = (G + 31) // 32
    return 40 * P + 8 * RW + 2 * 2 * 2500 + R * 44 + 48


def qnet_flops(n_act, B, hidden=512, in_dim=484, actions=5):
    """Dense MLP FLOPs: act forward over n_act rows + learn (online fwd, target fwd, backward dW+dX).
    in_dim 484: the live inputs of the 726 (channel 0 is identically zero, channel 5 a constant
    folded into the bias; csrc/qmlp.hip)."""
    fwd = 2 * (in_dim * hidden + hidden * (hidden // 2) + (hidden // 2) * actions)
    bwd = 2 * fwd - 2 * in_dim * hidden  # no dX for the input layer
    return n_act * fwd + B * (2 * fwd + bwd)


def cfg_name(args):
    """BASELINE.json configs: cfg2 64x64 x 8 robots, cfg3 128x128 x 16 (the headline), cfg4
    256x256 conv Q-net, cfg5 128x128 x 32 with prioritized replay."""
    if args.grid == 64 and args.robots == 8:
        return "cfg2"
    if args.grid == 256:
        return "cfg4"
    if args.robots == 32 and args.replay == "prioritized":
        return "cfg5"
    return "cfg3" if (args.grid, args.robots) == (128, 16) else f"custom {args.grid}x{args.grid} R{args.robots}"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=1300)
    ap.add_argument("--stagger", type=int, default=1200,
                    help="warmup step w force-resets envs with global id %% stagger == w, so the timed steps see "
                         "env ages spread over a whole episode (the stationary mix of a long run); 0 = off")
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--grid", type=int, default=128)
    ap.add_argument("--layouts", type=int, default=1,
                    help="K > 1: per-env layouts, K random variants of the synthetic layout (env e runs e %% K)")
    ap.add_argument("--people", type=int, default=2276)
    ap.add_argument("--robots", type=int, default=16)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--precision", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--qnet", choices=["mlp", "conv"], default="mlp",
                    help="conv: the reference's DQNNetwork (3 conv3x3 + fc stack) on the general MFMA GEMMs "
                         "(cfg4); mlp: the fused 726-512-256-5 kernels")
    ap.add_argument("--mode", choices=["train", "env"], default="train")
    ap.add_argument("--env-steps", type=int, default=100, help="extra env-only timed steps (0 = skip)")
    ap.add_argument("--strict-steps", type=int, default=100,
                    help="extra timed steps in the strict schedule after a lagged run (0 = skip)")
    ap.add_argument("--cpu-envs", type=int, default=2048)
    ap.add_argument("--cpu-steps", type=int, default=600)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--schedule", choices=["strict", "lagged"], default="lagged",
                    help="strict: act, env.step, push, learn (the reference's order); lagged: learn t samples "
                         "the ring before push t and overlaps env.step t (evacx.trainer.VecTrainer)")
    ap.add_argument("--replay", choices=["uniform", "prioritized"], default="uniform",
                    help="prioritized: GPU sum/min-tree proportional replay (cfg5; evacx.prio)")
    ap.add_argument("--replay-capacity", type=int, default=1 << 20)
    ap.add_argument("--groups", type=int, default=1,
                    help="env groups per GPU, each with its own act -> env.step -> push stream chain "
                         "(evacx.trainer._Group): one group's env.step tail overlaps the others' work")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r1", "env_traffic.json"),
                    help="PMC traffic record of env_step_kernel on this workload (tools/parse_prof.py)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer, make_allreduce_hook

    L = W = args.grid
    P, R, E = args.people, args.robots, args.envs
    spec = synthetic(L, W, R)
    layout_of = None
    if args.layouts > 1:  # per-env layouts: env e runs random layout e % K
        from evacx.env import LayoutSet
        from evacx.layout import random_layout
        lay = LayoutSet([DeviceLayout(build_tables(random_layout(L, W, R, 4242 + k)), P) for k in range(args.layouts)])
        layout_of = [(rank * E + e) % args.layouts for e in range(E)]
        tables = lay.tables
    else:
        tables = build_tables(spec)
        lay = DeviceLayout(tables, P)
    hook = make_allreduce_hook(dist, world) if dist is not None else None
    tr = VecTrainer(lay, E, env_offset=rank * E, kind=args.qnet, precision=args.precision, batch=args.batch,
                    grad_hook=hook,
                    lagged_learn=args.schedule == "lagged", replay=args.replay,
                    replay_capacity=args.replay_capacity, groups=args.groups if args.mode == "train" else 1,
                    layout_of=layout_of)
    env = tr.env

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ------------------------------------------------------------ warmup
    # Env ages are staggered over one episode length: a synchronised start would time
    # only one episode phase (per-step cost varies several-fold over an episode).
    gid = torch.arange(E, device="cuda") + rank * E
    S = args.stagger
    for w in range(args.warmup):
        force = (gid % S == w) if 0 < S and w < S else None
        if args.mode == "train":
            tr.step(extra_reset=force)
        else:
            env.step(torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32), auto_reset=True)
            if force is not None:
                env.reset(mask=force & ~env.done.bool())
    if args.mode == "train":
        tr.sync()
    barrier()

    # the CPU baseline continues from exactly this state (same envs, same episode phase)
    cpu_snap = None
    if rank == 0 and not args.no_cpu:
        cpu_snap = [env.host_state(i) for i in range(min(args.cpu_envs, E))]

    # ------------------------------------------------------- timed steps
    ev_env = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    ev_learn = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    rand_actions = torch.randint(0, 5, (args.steps, E * R), device="cuda", dtype=torch.int32)
    barrier()
    t0 = time.perf_counter()
    # HIP events bracket env.step on its own stream on every EV_EVERY-th step only: an
    # event record costs the stream a ~6 us gap (tools/gap_probe.py), which would
    # otherwise be charged to every timed step
    timed = [s for s in range(args.steps) if s % EV_EVERY == 0]
    for s in range(args.steps):
        ee = ev_env[s] if s % EV_EVERY == 0 else None
        el = ev_learn[s] if s % EV_EVERY == 0 else None
        if args.mode == "train":
            tr.step(ev_env=ee, ev_learn=el)
        else:
            env.compute_order()
            if ee is not None:
                ee[0].record()
            env.step(rand_actions[s], order=False, auto_reset=True)  # finished envs reset in the launch
            if ee is not None:
                ee[1].record()
    if args.mode == "train":
        tr.sync()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    env.check_err()
    kern_ms = float(np.mean([ev_env[s][0].elapsed_time(ev_env[s][1]) for s in timed]))
    learn_ms = (float(np.mean([ev_learn[s][0].elapsed_time(ev_learn[s][1]) for s in timed]))
                if args.mode == "train" else None)
    loss = float(tr.last_loss.item()) if tr.last_loss is not None else None

    # ------------------- the reference's strict order on the same state (extra)
    strict = None
    if args.mode == "train" and args.schedule == "lagged" and args.strict_steps > 0:
        tr.sync()
        tr.lagged = False
        for _ in range(20):
            tr.step()
        tr.sync()
        barrier()
        t1 = time.perf_counter()
        for _ in range(args.strict_steps):
            tr.step()
        tr.sync()
        barrier()
        strict = E * world * args.strict_steps / max_over_ranks(time.perf_counter() - t1)
        tr.lagged = True

    # --------------------------------------------- env-only rate (extra)
    env_only = None
    if args.env_steps > 0 and args.mode == "train":
        acts = torch.randint(0, 5, (args.env_steps, E * R), device="cuda", dtype=torch.int32)
        barrier()
        t1 = time.perf_counter()
        for s in range(args.env_steps):
            env.step(acts[s], auto_reset=True)
        barrier()
        env_only = E * world * args.env_steps / max_over_ranks(time.perf_counter() - t1)

    value = E * world * args.steps / elapsed
    G = (L + 2) * (W + 2)
    bpe = bytes_per_env_step(P, R, G)
    per_launch = E // args.groups if args.mode == "train" else E  # env.step launches of group 0 are timed
    achieved = bpe * per_launch / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic):
        # HBM bytes per launch from rocprofv3 PMC passes of this same workload (separate
        # --pmc FETCH_SIZE / WRITE_SIZE runs; cannot be collected inside the timed run)
        rec = json.load(open(args.traffic))
        if rec.get("kernel") == "env_step_kernel":
            traffic = rec["bytes_per_env_step"] * per_launch
    cpu = cpu_baseline(cpu_snap, env.lay.R, tables, P, args) if cpu_snap is not None else None
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "agent_transitions_per_s": value * R,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "stagger": args.stagger,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.mode == "env" else f"f64 env + {args.precision} Q-net",
            "data": "synthetic",
            "config": {
                "workload": (f"{cfg_name(args)} per-GPU share: {L}x{W} synthetic layout"
                             + (f" ({args.layouts} random per-env layouts)" if args.layouts > 1 else "")
                             + f", {P} people, {R} robots, {E} envs/GPU; "
                             + ("full training step: act + env.step + replay push + learn (B="
                                f"{args.batch}) + auto-reset" if args.mode == "train"
                                else "env.step + auto-reset, uniform random actions")),
                "envs_per_gpu": E, "grid": f"{L}x{W}", "people": P, "robots": R, "mode": args.mode,
                "batch": args.batch, "schedule": args.schedule if tr.fast is not None else "strict",
                "qnet": ("MLP 726-512-256-5" if args.qnet == "mlp"
                         else "DQNNetwork conv 6-32-64-128 + 15488-512-256-5"),
                "replay": args.replay, "groups": args.groups if args.mode == "train" else 1,
                "parallelism": f"data-parallel over {world} GPU(s): envs sharded, grad all-reduce (RCCL) per learn",
            },
            "strict_schedule_steps_per_s": strict,
            "env_only_steps_per_s": env_only,
            "env_step_kernel_ms": kern_ms,
            "learn_ms": learn_ms,
            "last_loss": loss,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "env_step_kernel",
                         "kernel_ms": kern_ms, "bytes_per_env_step": bpe, "env_steps_per_launch": per_launch,
                         "launches_timed": len(timed)},
            "cpu_baseline": cpu,
        }
        if learn_ms is not None and args.qnet == "mlp":
            fl = qnet_flops(0, args.batch)
            line["roofline_learn"] = {"bound": "mfma", "achieved": fl / (learn_ms * 1e-3) / 1e12,
                                      "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                                      "frac": fl / (learn_ms * 1e-3) / 1e12 / BF16_PEAK_TFLOPS}
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(snap, R, tables, P, args):
    """Oracle (C restatement, OpenMP over envs) on the host cores, started from the GPU
    state of the first cpu_envs envs at the beginning of the timed region (same episode
    phase), stepped with uniform random actions."""
    try:
        from oracle import oracle as orc
    except Exception as e:  # oracle not built: report, never fall back
        return {"error": f"oracle unavailable: {e}"}
    n = len(snap)
    olay = orc.Layout.from_tables(tables, P)
    envs = []
    for st in snap:
        oe = orc.Env(olay, thmap=False)
        oe.load_state(st)
        envs.append(oe)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    steps = args.cpu_steps
    acts = np.random.RandomState(0).randint(0, 5, size=(steps, n * R)).astype(np.int32)
    t0 = time.perf_counter()
    done_steps, _ = orc.run_batch(olay, envs, steps, acts, nthreads=cores)
    dt = time.perf_counter() - t0
    return {"value": done_steps / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{n} envs x {steps} env.steps of the same workload from the GPU's warmed-up state "
                      f"(env.step only, no learner), OpenMP {cores} threads, {dt:.2f}s wall, "
                      f"{dt * cores:.1f} core-s"}


if __name__ == "__main__":
    main()
