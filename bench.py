#!/usr/bin/env python3
"""Benchmark of the evacuation hot path on MI355X (contract: see README/DESIGN.md).

Default workload (BASELINE.json metric, cfg3 per-GPU share): 128x128 synthetic
layout, 2276 people and 16 robots per env, 4096 envs per GPU, uniform random
actions, auto-reset, weak scaling over GPUs (env ids are global, seeds
1234 + global env id). One "step" = one vectorised env.step over all envs
(env mode) or env.step + act forward + replay push + one learn step (train mode).

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
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def bytes_per_env_step(P, R, G):
    """Algorithmic HBM bytes of one env-step of env_step_kernel:
    people r+w (pk 4 + health 8 + acc 8) x2, rmap bitmap r+w, two MT19937 states r+w,
    per robot action 4 + position r/w 8 + compact obs 32, per-env scalars 48.
    Shared read-only tables (floor, danger, valid bits) are L2/MALL-resident and excluded."""
    RW = (G + 31) // 32
    return 40 * P + 8 * RW + 2 * 2 * 2500 + R * 44 + 48


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--grid", type=int, default=128)
    ap.add_argument("--people", type=int, default=2276)
    ap.add_argument("--robots", type=int, default=16)
    ap.add_argument("--mode", choices=["env"], default="env")
    ap.add_argument("--cpu-envs", type=int, default=512)
    ap.add_argument("--cpu-steps", type=int, default=100)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-kernel-events", action="store_true", default=True)
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

    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic

    L = W = args.grid
    P, R, E = args.people, args.robots, args.envs
    spec = synthetic(L, W, R)
    tables = build_tables(spec)
    lay = DeviceLayout(tables, P)
    env = VecEnv(lay, E)
    env.seed([1234 + rank * E + i for i in range(E)])
    env.reset()

    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234 + rank)
    nact = args.warmup + args.steps
    actions = torch.randint(0, 5, (nact, E * R), generator=gen, device="cuda", dtype=torch.int32)

    def step(i):
        env.step(actions[i])
        env.reset(mask=env.done)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()

    # per-launch kernel time of the dominant kernel (env_step) on its own stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        a, b = ev[s]
        a.record()
        env.step(actions[args.warmup + s])
        b.record()
        env.reset(mask=env.done)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    env.check_err()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if dist is not None:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    env_steps = E * world * args.steps
    value = env_steps / elapsed
    G = (L + 2) * (W + 2)
    bpe = bytes_per_env_step(P, R, G)
    achieved = bpe * E / (kern_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(env, tables, P, args, actions)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "agent_transitions_per_s": value * R,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"cfg3 per-GPU share: {L}x{W} synthetic layout, {P} people, {R} robots, "
                                   f"{E} envs/GPU, uniform random actions, auto-reset (env.step + reset)",
                       "envs_per_gpu": E, "grid": f"{L}x{W}", "people": P, "robots": R, "mode": args.mode,
                       "parallelism": f"envs sharded over {world} GPU(s), no collective in env mode"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "env_step_kernel", "kernel_ms": kern_ms, "bytes_per_env_step": bpe},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(env, tables, P, args, actions):
    """Oracle (C restatement, OpenMP over envs) on the host cores, continuing from the
    GPU's warmed-up state of the first cpu_envs envs with the same actions."""
    try:
        from oracle import oracle as orc
    except Exception as e:  # oracle not built: report, never fall back
        return {"error": f"oracle unavailable: {e}"}
    n = min(args.cpu_envs, env.E)
    olay = orc.Layout.from_tables(tables, P)
    envs = []
    for i in range(n):
        oe = orc.Env(olay, thmap=False)
        oe.load_state(env.host_state(i))
        envs.append(oe)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    R = env.lay.R
    steps = args.cpu_steps
    acts = torch.randint(0, 5, (steps, n * R), dtype=torch.int32).numpy()
    t0 = time.perf_counter()
    done_steps, _ = orc.run_batch(olay, envs, steps, acts, nthreads=cores)
    dt = time.perf_counter() - t0
    return {"value": done_steps / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{n} envs x {steps} steps of the same workload from the GPU's warmed-up state, "
                      f"OpenMP {cores} threads, {dt:.2f}s wall"}


if __name__ == "__main__":
    main()
