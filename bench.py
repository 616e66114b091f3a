#!/usr/bin/env python3
"""Benchmark of the evacuation RL hot path on MI355X.

Workload (BASELINE.json metric; configs[2] as stated, which fits one MI355X): synthetic
128x128 layout, 2276 people and 16 robots per env, 32768 envs per GPU (weak scaling: N GPUs
step N x 32768 envs; env ids global, seeds 1234 + global env id), uniform-init MLP Q-net,
learn batch = envs per GPU (one sampled transition per env-step, as the 8-GPU data-parallel
run's global batch 8 x 4096), replay 16 steps of pushes per GPU (2^23 transitions), gradient
all-reduce over RCCL when world > 1. --envs 4096 --batch 4096 is the per-GPU share of the
8-GPU data-parallel run.
One timed "step" = one full vectorised training step in the reference's order
(DQNAgent act -> env.step -> remember -> learn, runners/train_dqn.py:94-116):
act (Q forward for E*R robots + epsilon-greedy) -> env.step (all E envs, finished
envs auto-reset inside the launch) -> replay push (E*R transitions) -> one learn
step (sample, online+target forward, TD loss, backward, [all-reduce], clip+Adam).

Episode phase. The cost of an env-step varies several-fold over an episode (all
2276 persons in play at its start, a few at its end), so the phase the timed steps
see is part of the workload and is built explicitly, independent of --warmup:
  --phase stationary (default): an env-only preparation of --age-steps steps
     (uniform random actions) force-resets env g at preparation step g % --stagger,
     so env ages are spread uniformly over one episode length -- the stationary mix
     of a long training run;
  --phase start: the same preparation, then every env is reset (fresh people, the
     fire kept, as EvacuationEnv.reset does): all envs at the start of an episode.
The start-of-episode rate is also reported beside the stationary value
(start_phase), from a full reset after the timed steps.

value = env-steps/s of the whole job (E * n_gpus * steps / time) at the headline
schedule and precision; the JSON line also carries agent-transitions/s (x R), the
other schedule's rate, the env-only rate, the roofline of the dominant kernel
(env_step_kernel, HBM-bound) and the CPU baseline. Prints ONE JSON line on rank 0.
"""
import argparse
import glob
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dqn-marl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env steps/sec + agent-transitions/sec (whole node), 128x128 grid, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (spec); f32 via bf16x3 split runs on the same pipe
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


def learn_flops_executed(B, tab_on, tab_tg, stat_rows, hidden=512, in_dim=484, occ=121, actions=5):
    """f32-equivalent FLOPs the fused learn chain EXECUTES for one learn step (csrc/qmlp.hip): a forward
    row whose fc1 starts from the per-centre act table (tab_on / tab_tg: the fraction of the batch's
    online / target rows that take it) contracts only fc1's 121 occupancy inputs, the others all 484;
    fc2, fc3 for every row; the backward dW3 + dH2, dW2 + dH1 and dW1 over all 484 inputs (no dX for
    the input layer); and the rebuild of the online net's table after the update (stat_rows centres x
    the full fc1 at zero occupancy)."""
    h2 = hidden // 2
    fc23 = hidden * h2 + h2 * actions
    row = lambda frac: frac * 2 * (occ * hidden + fc23) + (1 - frac) * 2 * (in_dim * hidden + fc23)  # noqa: E731
    bwd = 2 * (2 * h2 * actions + 2 * hidden * h2 + in_dim * hidden)
    return B * (row(tab_on) + row(tab_tg) + bwd) + stat_rows * 2 * in_dim * hidden


def counter_record(kind, phase, per_launch, L, P, R):
    """The newest SQ counter record (tools/env_counters.py via tools/gpu_r6_counters.sh) of env_step_kernel
    on exactly this workload: phase, envs per launch, grid, people and robots."""
    for r in ("r6",):
        for q in sorted(glob.glob(os.path.join(ROOT, "profiles", r, f"{kind}_*.json"))):
            try:
                rec = json.load(open(q))
            except (OSError, ValueError):
                continue
            if (rec.get("kernel") == "env_step_kernel" and rec.get("phase") == phase and rec.get("envs") == per_launch
                    and rec.get("grid") == [L, L] and rec.get("people") == P and rec.get("robots") == R
                    and rec.get("sq_insts_valu_per_wave") and rec.get("clock_ghz")):
                return rec, os.path.relpath(q, ROOT)
    return None, None


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
    ap.add_argument("--warmup", type=int, default=10, help="untimed training steps after the preparation")
    ap.add_argument("--phase", choices=["stationary", "start"], default="stationary",
                    help="episode phase of the timed steps (module docstring)")
    ap.add_argument("--age-steps", type=int, default=1300,
                    help="env-only preparation steps that spread env ages over an episode (before --warmup)")
    ap.add_argument("--stagger", type=int, default=1200,
                    help="preparation step w force-resets envs with global id %% stagger == w (0 = no stagger)")
    ap.add_argument("--envs", type=int, default=32768,
                    help="envs PER GPU (weak scaling: N GPUs step N x envs); see --envs-total")
    ap.add_argument("--envs-total", type=int, default=0,
                    help="envs of the WHOLE job, split evenly over the ranks (overrides --envs; strong-scaling "
                         "reading)")
    ap.add_argument("--total-reading", type=int, default=32768,
                    help="extra (N > 1 only): also time the training step with this many envs for the whole job "
                         "(BASELINE.json configs[2] read as 32768 envs over all GPUs: 32768 / N per GPU); 0 = skip")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend when WORLD_SIZE > 1 (nccl = RCCL over xGMI; gloo: CPU tests, "
                         "several ranks on one GPU)")
    ap.add_argument("--grid", type=int, default=128)
    ap.add_argument("--layouts", type=int, default=1,
                    help="K > 1: per-env layouts, K random variants of the synthetic layout (env e runs e %% K)")
    ap.add_argument("--people", type=int, default=2276)
    ap.add_argument("--robots", type=int, default=16)
    ap.add_argument("--batch", type=int, default=0, help="learn batch (0: = envs per GPU)")
    ap.add_argument("--precision", choices=["bf16", "f32"], default="f32",
                    help="Q-net arithmetic: f32 (the reference's; fused kernels with bf16x3-split MFMA operands) "
                         "or bf16")
    ap.add_argument("--qnet", choices=["mlp", "conv"], default="mlp",
                    help="conv: the reference's DQNNetwork (3 conv3x3 + fc stack) on the general MFMA GEMMs "
                         "(cfg4); mlp: the fused 726-512-256-5 kernels")
    ap.add_argument("--mode", choices=["train", "env"], default="train")
    ap.add_argument("--env-steps", type=int, default=100, help="extra env-only timed steps (0 = skip)")
    ap.add_argument("--other-steps", type=int, default=100,
                    help="extra timed steps in the other schedule (lagged when strict is the headline; 0 = skip)")
    ap.add_argument("--start-steps", type=int, default=20,
                    help="extra: timed training steps right after a full reset (start of episode; 0 = skip)")
    ap.add_argument("--cpu-envs", type=int, default=1024)
    ap.add_argument("--cpu-steps", type=int, default=600)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--schedule", choices=["strict", "lagged"], default="strict",
                    help="strict: act, env.step, push, learn (the reference's order); lagged: learn t samples "
                         "the ring before push t and overlaps env.step t (evacx.trainer.VecTrainer)")
    ap.add_argument("--replay", choices=["uniform", "prioritized"], default="uniform",
                    help="prioritized: GPU sum/min-tree proportional replay (cfg5; evacx.prio)")
    ap.add_argument("--replay-capacity", type=int, default=0,
                    help="transitions per GPU (0: the power of two >= 16 steps of pushes, envs x robots x 16)")
    ap.add_argument("--nets", choices=["shared", "per_robot", "qmix"], default="shared",
                    help="per_robot: every robot index has its own Q-network, memory and optimizer (SURVEY F3; "
                         "grouped launches, batch / robots transitions per net); qmix: those nets under a QMIX mixer "
                         "(batch / robots joint env-steps)")
    ap.add_argument("--act-table", choices=["auto", "on", "off"], default="auto",
                    help="x3 act table path (the per-centre table of fc1's static features, rebuilt every "
                         "update); auto: the trainer's choice")
    ap.add_argument("--groups", type=int, default=1,
                    help="env groups per GPU, each with its own act -> env.step -> push stream chain "
                         "(evacx.trainer._Group): one group's env.step tail overlaps the others' work")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic record of env_step_kernel on this workload and phase (tools/parse_prof.py); "
                         "default: the newest profiles/r*/ env_counters_<phase>*.json or env_traffic_<phase>*.json "
                         "record of this workload")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.envs_total > 0:
        if args.envs_total % world:
            ap.error("--envs-total must be a multiple of the world size")
        args.envs = args.envs_total // world
    if args.batch <= 0:
        args.batch = args.envs
    args.auto_capacity = args.replay_capacity <= 0
    if args.auto_capacity:
        args.replay_capacity = replay_capacity_for(args.envs, args.robots)
    return args


def replay_capacity_for(E, R):
    """The default ring: the power of two >= 16 steps of pushes (E envs x R robots x 16)."""
    c = 1
    while c < 16 * E * R:
        c <<= 1
    return c


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def host_threads():
    """Threads the CPU baseline may use: every core of this process's affinity set, capped
    by OMP_NUM_THREADS when the launcher sets it (a GPU box's per-GPU CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; with gloo, ranks beyond the visible GPUs share them (tests on one GPU)
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")

    from evacx.env import DeviceLayout
    from evacx.layout import build_tables_device, synthetic
    from evacx.trainer import VecTrainer, make_allreduce_hook

    L = W = args.grid
    P, R, E = args.people, args.robots, args.envs
    spec = synthetic(L, W, R)
    layout_of = None
    if args.layouts > 1:  # per-env layouts: env e runs random layout e % K
        from evacx.env import LayoutSet
        from evacx.layout import random_layout
        # floor fields of all K layouts in one device launch
        lay_tables = build_tables_device([random_layout(L, W, R, 4242 + k) for k in range(args.layouts)])
        lay = LayoutSet([DeviceLayout(t, P) for t in lay_tables])
        layout_of = [(rank * E + e) % args.layouts for e in range(E)]
    else:
        lay_tables = build_tables_device([spec])
        lay = DeviceLayout(lay_tables[0], P)
    hook = make_allreduce_hook(dist, world) if dist is not None else None

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

    def build(E, batch):
        """The trainer for E envs per rank (global env ids rank * E + e), prepared to the episode
        phase: env-only steps (uniform random actions) where preparation step w force-resets the
        envs with global id % stagger == w, spreading env ages over one episode length."""
        cap = replay_capacity_for(E, R) if args.auto_capacity else args.replay_capacity
        tr = VecTrainer(lay, E, env_offset=rank * E, kind=args.qnet, precision=args.precision, batch=batch,
                        grad_hook=hook,
                        lagged_learn=args.schedule == "lagged", replay=args.replay,
                        replay_capacity=cap, groups=args.groups if args.mode == "train" else 1,
                        layout_of=layout_of, world_envs=E * world, nets=args.nets,
                        act_table=None if args.act_table == "auto" else args.act_table == "on")
        env = tr.env
        gid = torch.arange(E, device="cuda") + rank * E
        S = args.stagger
        prep_acts = torch.empty(E * R, device="cuda", dtype=torch.int32)
        g = torch.Generator(device="cuda").manual_seed(4321 + rank)
        for w in range(args.age_steps):
            if rank == 0 and w % 200 == 0:  # progress on stderr (long profiled runs)
                print(f"preparation step {w}/{args.age_steps} ({E} envs per rank)", file=sys.stderr, flush=True)
            torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g, out=prep_acts)
            env.step(prep_acts, auto_reset=True)
            if 0 < S and w < S:
                force = (gid % S == w) & ~env.done.bool()
                env.reset(mask=force)
        if args.phase == "start":
            env.reset()  # every env at the start of an episode (people fresh, fire kept)
        barrier()
        return tr, env

    S = args.stagger
    tr, env = build(E, args.batch)
    lagged_ok = tr.fast is not None  # the lagged schedule needs the fused MLP path
    schedule = args.schedule if lagged_ok else "strict"

    def timed_train(n, ev_env=None, ev_learn=None, ev_act=None):
        barrier()
        t0 = time.perf_counter()
        for s in range(n):
            if args.mode == "train":
                tr.step(ev_env=None if ev_env is None or s % EV_EVERY else ev_env[s],
                        ev_learn=None if ev_learn is None or s % EV_EVERY else ev_learn[s],
                        ev_act=None if ev_act is None or s % EV_EVERY else ev_act[s])
            else:
                env.compute_order()
                if ev_env is not None and s % EV_EVERY == 0:
                    ev_env[s][0].record()
                env.step(acts_env[s % acts_env.shape[0]], order=False, auto_reset=True)
                if ev_env is not None and s % EV_EVERY == 0:
                    ev_env[s][1].record()
        if args.mode == "train":
            tr.sync()
        barrier()
        return max_over_ranks(time.perf_counter() - t0)

    def ev_pairs(n):
        return [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]

    def ev_mean(evs, n):
        return float(np.mean([evs[s][0].elapsed_time(evs[s][1]) for s in range(n) if s % EV_EVERY == 0]))

    # the CPU baseline continues from this state (same envs, same episode phase). Taken before the
    # warm-up, so the timed steps follow the warm-up at once: a host copy between them left the
    # GPU idle long enough to start the timed region at lower clocks (16.6 vs 17.6 M env-steps/s
    # measured on one box)
    cpu_snap = None
    if rank == 0 and not args.no_cpu:
        cpu_snap = [(env.host_state(i), layout_of[i] if layout_of else 0) for i in range(min(args.cpu_envs, E))]

    # ----------------------------------------------------------------- warmup
    acts_env = torch.randint(0, 5, (max(args.steps, args.warmup, 1), E * R), device="cuda", dtype=torch.int32)
    timed_train(args.warmup)

    # ------------------------------------------------------------ timed steps
    # no instrumentation inside the timed region: an event record costs the stream a ~6 us gap
    # (tools/gap_probe.py), 4 records per instrumented step -- 1.6 % of cfg2's step at one
    # instrumented step in EV_EVERY
    elapsed = timed_train(args.steps)
    env.check_err()
    loss = float(tr.last_loss.float().mean().item()) if tr.last_loss is not None else None
    value = E * world * args.steps / elapsed
    # the kernel / learn times: a second pass of the same length right after (same episode phase),
    # HIP events bracketing env.step and the learn step on every EV_EVERY-th step
    ev_env, ev_learn, ev_act = ev_pairs(args.steps), ev_pairs(args.steps), ev_pairs(args.steps)
    train = args.mode == "train"
    timed_train(args.steps, ev_env, ev_learn if train else None, ev_act if train else None)
    env.check_err()
    kern_ms = ev_mean(ev_env, args.steps)
    learn_ms = ev_mean(ev_learn, args.steps) if train else None
    act_ms = ev_mean(ev_act, args.steps) if train else None
    # the act's rows on the table path (fire step at the layout's last: fc1 = table + occupancy columns)
    act_tab = None
    if train and tr.fast is not None and getattr(tr.fast, "_static", None) is not None:
        act_tab = float((env.obs.view(-1, 8)[:, 6] >= int(tr.lay.c.t_max)).float().mean().item())

    # ------------------------------- the other schedule on the same state (extra)
    other = None
    if args.mode == "train" and lagged_ok and args.other_steps > 0:
        tr.sync()
        tr.lagged = schedule == "strict"
        timed_train(10)
        other = {"schedule": "lagged" if tr.lagged else "strict",
                 "steps_per_s": E * world * args.other_steps / timed_train(args.other_steps)}
        tr.lagged = schedule == "lagged"

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

    # ------------------------- start of episode: every env freshly reset (extra)
    start = None
    if args.start_steps > 0 and args.phase == "stationary":
        tr.sync()
        env.reset()
        ev_s = ev_pairs(args.start_steps)
        dt = timed_train(args.start_steps, ev_s)
        start = {"steps_per_s": E * world * args.start_steps / dt, "env_step_kernel_ms": ev_mean(ev_s, args.start_steps),
                 "steps": args.start_steps,
                 "what": "every env reset (all persons in play), then the timed training steps"}

    # ------ the learn step alone (extra: its MFMA roofline). The last reading on the headline
    # trainer (its six extra learn steps move the weights, Adam, epsilon); without the gradient
    # all-reduce, so it is the learn chain's own time at any world size
    learn_alone_ms = None
    if args.mode == "train" and tr.fast is not None and tr.replay.size >= args.batch:
        tr.sync()
        hook_saved, tr.learner.grad_hook = tr.learner.grad_hook, None
        ev_l = ev_pairs(6)
        for i in range(6):
            ev_l[i][0].record()
            tr.learn()
            ev_l[i][1].record()
        torch.cuda.synchronize()
        tr.learner.grad_hook = hook_saved
        learn_alone_ms = float(np.mean([ev_l[i][0].elapsed_time(ev_l[i][1]) for i in range(1, 6)]))
    # which forward rows of the learn batch start fc1 from an act table (the fused act kernel's table
    # path: the online / target forwards at B >= 32768, rows at the layout's last fire step, whole
    # 64-row tiles), from the last drawn batch -- for the executed-FLOP basis of roofline_learn
    learn_tab = None
    if args.mode == "train" and tr.fast is not None and tr.learner is not None and not tr.per_robot:
        st = getattr(tr.fast, "_static", None)
        stat_rows = int(st[1].shape[0]) if st is not None else 0
        fr = [0.0, 0.0]
        if st is not None and args.batch >= 32768:
            t_max = int(tr.lay.c.t_max)
            for i, key in enumerate(("s", "s2")):
                fs = tr.samp[key].view(-1, 8)[:args.batch, 6]
                tile_all = (fs >= t_max).view(-1, 64).all(dim=1) if args.batch % 64 == 0 else None
                fr[i] = float(tile_all.float().mean().item()) if tile_all is not None else 0.0
            if getattr(tr.learner, "fast_t", None) is None or getattr(tr.learner.fast_t, "_static", None) is None:
                fr[1] = 0.0
        learn_tab = (fr[0], fr[1], stat_rows)

    # ---------- BASELINE configs[2] read as envs for the whole job (extra, N > 1 only)
    total = None
    Et = args.total_reading // world if args.total_reading > 0 and args.total_reading % world == 0 else 0
    if args.mode == "train" and world > 1 and Et > 0 and Et != E and args.envs_total == 0:
        tr.sync()
        tr = env = None  # free the headline's state first
        torch.cuda.empty_cache()
        tr, env = build(Et, Et)
        timed_train(max(args.warmup, 3))
        n_t = max(5, args.steps // 2)
        dt = timed_train(n_t)
        total = {"envs_total": Et * world, "envs_per_gpu": Et, "batch_per_gpu": Et, "steps": n_t,
                 "steps_per_s": Et * world * n_t / dt, "agent_transitions_per_s": Et * world * n_t / dt * R,
                 "ms_per_step": 1e3 * dt / n_t,
                 "what": f"BASELINE.json configs[2] read as {Et * world} envs for the whole {world}-GPU job "
                         f"({Et} per GPU, learn batch {Et} per GPU), same phase preparation and schedule"}

    G = (L + 2) * (W + 2)
    bpe = bytes_per_env_step(P, R, G)
    per_launch = E // args.groups if args.mode == "train" else E  # env.step launches of group 0 are timed
    achieved = bpe * per_launch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src, traffic_corr = None, None, None
    def traffic_match(q):  # a PMC record of this kernel, phase, launch size and grid
        try:
            rec = json.load(open(q))
        except (OSError, ValueError):
            return False
        return (rec.get("kernel") == "env_step_kernel" and rec.get("envs") in (None, per_launch)
                and rec.get("grid", [L, W]) == [L, W] and rec.get("people", P) == P and rec.get("robots", R) == R)
    tpath = args.traffic or next((q for r in ("r6", "r5", "r4", "r3", "r2")
                                  for pat in (f"env_counters_{args.phase}*.json", f"env_traffic_{args.phase}*.json")
                                  for q in sorted(glob.glob(os.path.join(ROOT, "profiles", r, pat)))
                                  if traffic_match(q)), "")
    if os.path.exists(tpath):
        # HBM bytes per launch from rocprofv3 PMC passes of this same workload and phase
        # (separate --pmc FETCH_SIZE / WRITE_SIZE runs; cannot be collected inside the timed run)
        rec = json.load(open(tpath))
        if rec.get("kernel") == "env_step_kernel" and rec.get("envs") in (None, per_launch):
            # raw FETCH + WRITE: the x2 FETCH correction of MI355X_MICROARCH.md holds for 16-B/lane
            # streaming reads, and this kernel's loads are 4-8 B per lane; the corrected figure rides along
            traffic = rec.get("bytes_per_env_step_raw", rec["bytes_per_env_step"]) * per_launch
            traffic_corr = rec["bytes_per_env_step"] * per_launch
            traffic_src = os.path.relpath(tpath, ROOT)
    # the issue roofline of the same kernel: VALU + SALU instructions per wave x waves
    # per launch (SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_WAVES, one --pmc pass of this workload) against one
    # instruction per SIMD per cycle (256 CUs x 4 SIMDs x the clock the GRBM pass measured) over the
    # launch time measured here; valu_pipe_frac prices a wave64 VALU at 2 cycles of its SIMD-32
    # (MI355X_MICROARCH.md, cycle constants)
    roof_hbm = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                "traffic_basis": "raw FETCH_SIZE + WRITE_SIZE bytes per launch (PMC)",
                "traffic_fetch_x2": traffic_corr,
                "frac_traffic": (traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                "frac_basis": "algorithmic bytes (bytes_per_env_step x env-steps per launch) / kernel_ms / peak; "
                              "frac_traffic: the PMC bytes the kernel actually moved, same time",
                "kernel": "env_step_kernel", "kernel_ms": kern_ms, "bytes_per_env_step": bpe,
                "env_steps_per_launch": per_launch,
                "launches_timed": len([s for s in range(args.steps) if s % EV_EVERY == 0])}
    roof_issue = None
    srec, ssrc = counter_record("env_counters", args.phase, per_launch, L, P, R)
    if srec is not None:
        waves = srec["waves"]
        insts = (srec["sq_insts_valu_per_wave"] + srec["sq_insts_salu_per_wave"]) * waves
        clk = min(srec["clock_ghz"], 2.4) * 1e9  # GRBM reads high on dispatches under ~0.3 ms: at most the 2.4 GHz peak
        t = kern_ms * 1e-3
        roof_issue = {"bound": "issue", "achieved": insts / t / 1e9, "peak": 1024 * clk / 1e9, "unit": "Ginst/s",
                      "frac": insts / (1024 * clk * t),
                      "valu_pipe_frac": srec["sq_insts_valu_per_wave"] * waves * 2 / (1024 * clk * t),
                      "valu_per_wave": srec["sq_insts_valu_per_wave"], "salu_per_wave": srec["sq_insts_salu_per_wave"],
                      "waves_per_launch": waves, "clock_ghz": min(srec["clock_ghz"], 2.4), "kernel_ms": kern_ms,
                      "sq_active_inst_any_frac": srec.get("sq_active_inst_any_frac"),
                      "sq_wait_any_frac": srec.get("sq_wait_any_frac"), "source": ssrc,
                      "basis": "(VALU + SALU instructions per wave) x waves / (256 CUs x 4 SIMDs x clock x kernel_ms): "
                               "one instruction per SIMD per cycle"}
    # the binding roof: the larger of the measured-traffic HBM fraction and the issue fraction
    roof = roof_hbm
    if roof_issue is not None and roof_issue["frac"] > (roof_hbm["frac_traffic"] or 0.0):
        roof = dict(roof_issue, traffic=traffic, traffic_source=traffic_src)
    cpu = None
    if cpu_snap is not None:
        cpu = cpu_baseline(cpu_snap, env.lay.R, lay_tables, P, args, E)
    if rank == 0:
        prec = args.precision
        qdesc = ("f32-accurate Q-net: x3 (bf16 hi+lo operand pairs on the bf16 MFMA, f32 accumulation; "
                 "Q and loss within rtol 2e-4 of torch fp32)" if tr.q_arith == "x3" else f"{tr.q_arith} Q-net")
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
            "dtype": "f64" if args.mode == "env" else f"f64 env + {qdesc}",
            "data": "synthetic",
            "config": {
                "workload": (f"{cfg_name(args)}{' (BASELINE.json configs[2] as stated)' if E == 32768 and (L, R) == (128, 16) else ''}"
                             f" per GPU: {L}x{W} synthetic layout"
                             + (f" ({args.layouts} random per-env layouts)" if args.layouts > 1 else "")
                             + f", {P} people, {R} robots, {E} envs/GPU; "
                             + (f"full training step ({schedule} schedule): act + env.step + replay push + learn "
                                f"(B={args.batch}) + auto-reset" if args.mode == "train"
                                else "env.step + auto-reset, uniform random actions")
                             + ("; episode phase: stationary mix (env ages spread uniformly over "
                                f"{S} steps by a {args.age_steps}-step env-only preparation)"
                                if args.phase == "stationary" else
                                "; episode phase: start (every env freshly reset before the timed steps)")),
                "episode_phase": args.phase, "age_steps": args.age_steps, "stagger": S,
                "envs_per_gpu": E, "envs_total": E * world,
                "baseline_mapping": ("BASELINE.json configs[2] (32768 envs x 16 agents, 128x128) is run as "
                                     f"{E} envs PER GPU (weak scaling: {E * world} envs over {world} GPU(s)), learn "
                                     f"batch {args.batch} per GPU; the whole-job-32768 reading is "
                                     "total_envs_reading (N > 1)") if (L, R) == (128, 16) else None, "grid": f"{L}x{W}", "people": P, "robots": R, "mode": args.mode,
                "batch": args.batch, "replay_capacity": args.replay_capacity, "schedule": schedule, "precision": prec,
                "q_arithmetic": tr.q_arith,
                "replay_sampling": ("uniform without replacement (random.sample semantics: keyed Feistel permutation "
                                    "per learn step)") if args.replay == "uniform" else "proportional prioritized",
                "qnet": ("MLP 726-512-256-5" if args.qnet == "mlp"
                         else "DQNNetwork conv 6-32-64-128 + 15488-512-256-5"),
                "replay": args.replay, "groups": args.groups if args.mode == "train" else 1, "nets": args.nets,
                "parallelism": (f"data-parallel over {world} GPU(s): envs sharded by global id, grad all-reduce "
                                f"({'RCCL' if args.dist_backend == 'nccl' else 'gloo'}) per learn"
                                if world > 1 else "1 GPU"),
                "dist_backend": args.dist_backend if world > 1 else None,
            },
            "total_envs_reading": total,
            "other_schedule": other,
            "env_only_steps_per_s": env_only,
            "start_phase": start,
            "env_step_kernel_ms": kern_ms,
            "learn_ms": learn_ms,
            "learn_ms_what": "the learn step on the training stream (every 5th step of the instrumented pass "
                             "that follows the timed steps)",
            "learn_alone_ms": learn_alone_ms,
            "last_loss": loss,
            "roofline": roof,
            "roofline_hbm": roof_hbm,
            "roofline_issue": roof_issue,
            "roofline_binding": ("the larger of roofline_hbm.frac_traffic (PMC bytes moved) and roofline_issue.frac "
                                 "(SQ instruction counts) on this workload; roofline_hbm.frac is on the "
                                 "algorithmic bytes") if roof_issue is not None else "no SQ record for this workload",
            "cpu_baseline": cpu,
        }
        if act_ms is not None and args.qnet == "mlp" and tr.q_arith == "x3" and not tr.per_robot:
            rows = E * R
            tf = act_tab or 0.0
            # bf16 MFMA products the x3 act issues per row: fc1 (table rows: the 128 occupancy columns,
            # hi + lo weights; others: 640 hi*hi + 512 hi*lo of K), fc2 3 x 512 K, fc3 (5 actions padded to
            # the 32-row MFMA tile) 3 x 256 K; f32-equivalent: the reference's products, fc1 over the 121
            # occupancy inputs on the table path, else the 484 live inputs
            prod = 2 * (tf * 512 * 128 * 2 + (1 - tf) * 512 * (640 + 512) + 256 * 512 * 3 + 32 * 256 * 3)
            f32eq = 2 * (tf * 121 * 512 + (1 - tf) * 484 * 512 + 512 * 256 + 256 * 5)
            ach = rows * prod / (act_ms * 1e-3) / 1e12
            line["roofline_act"] = {"bound": "mfma", "achieved": ach, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                                    "frac": ach / BF16_PEAK_TFLOPS, "act_ms": act_ms, "rows": rows,
                                    "table_rows": tf,
                                    "frac_f32eq": rows * f32eq / (act_ms * 1e-3) / 1e12 / BF16_PEAK_TFLOPS,
                                    "flops_basis": "bf16 MFMA products issued by the x3 act (frac) and the reference's "
                                                   "f32 products (frac_f32eq) per row x rows / act_ms (HIP events around "
                                                   "the act launch(es), every 5th step of the instrumented pass)"}
            if rows == 524288 and tf >= 0.99:  # cfg3's act: the PMC pass on this workload (clock and MFMA-busy)
                clk = 2.03  # GRBM_GUI_ACTIVE / duration of qact3p_kernel, profiles/r6/counters_r6.md
                line["roofline_act"].update({
                    "clock_ghz_pmc": clk, "mfma_busy_pmc": 0.522,
                    "frac_at_clock": ach / (BF16_PEAK_TFLOPS * clk / 2.4),
                    "pmc_source": "profiles/r6/counters_r6.md (qact3p_kernel: SQ_VALU_MFMA_BUSY_CYCLES, GRBM clock)",
                    "clock_note": "the sustained MFMA load holds the act at ~2.03 GHz (2.4 GHz peak): frac_at_clock "
                                  "prices the same products against the peak at that clock"})
        lm = learn_alone_ms if learn_alone_ms is not None else learn_ms
        if lm is not None and args.qnet == "mlp" and learn_tab is not None:
            fl = learn_flops_executed(args.batch, *learn_tab)
            fd = qnet_flops(0, args.batch)
            line["roofline_learn"] = {"bound": "mfma", "achieved": fl / (lm * 1e-3) / 1e12,
                                      "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                                      "frac": fl / (lm * 1e-3) / 1e12 / BF16_PEAK_TFLOPS, "learn_ms": lm,
                                      "flops": fl, "flops_dense": fd,
                                      "frac_dense": fd / (lm * 1e-3) / 1e12 / BF16_PEAK_TFLOPS,
                                      "table_rows": {"online": learn_tab[0], "target": learn_tab[1],
                                                     "rebuild_centres": learn_tab[2]},
                                      "flops_basis": "f32-equivalent FLOPs the learn chain executes (learn_flops_executed: "
                                                     "fc1 over the 121 occupancy inputs for rows that start from the act "
                                                     "table, 484 otherwise, plus the table rebuild); frac_dense: every "
                                                     "row over all 484 inputs, no rebuild. B rows, timed alone, no "
                                                     "all-reduce. The x3 arithmetic issues 2-3 bf16 MFMA products per "
                                                     "f32 product"}
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def cpu_learner_ms(args, threads):
    """The reference's learn step (agents/dqn_agent.py:126-168) and act forward for the MLP
    variant, in torch on the host cores: ms per learn at B=batch, ms per act row."""
    import torch.nn as nn
    torch.set_num_threads(threads)
    net = nn.Sequential(nn.Linear(726, 512), nn.ReLU(), nn.Dropout(0.2), nn.Linear(512, 256), nn.ReLU(),
                        nn.Linear(256, 5))
    tgt = nn.Sequential(nn.Linear(726, 512), nn.ReLU(), nn.Dropout(0.2), nn.Linear(512, 256), nn.ReLU(),
                        nn.Linear(256, 5))
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    B = args.batch
    s, s2 = torch.rand(B, 726), torch.rand(B, 726)
    a = torch.randint(0, 5, (B,))
    r, d = torch.rand(B), torch.zeros(B, dtype=torch.bool)

    def learn():
        q = net(s).gather(1, a.unsqueeze(1))
        with torch.no_grad():
            y = r + 0.99 * tgt(s2).max(1)[0] * ~d
        loss = nn.functional.mse_loss(q.squeeze(), y)
        opt.zero_grad()
        loss.backward()
        nn.utils.clip_grad_norm_(net.parameters(), 1.0)
        opt.step()

    n_act = 8192
    xa = torch.rand(n_act, 726)
    for _ in range(2):
        learn()
        with torch.no_grad():
            net(xa).argmax(1)
    t0 = time.perf_counter()
    for _ in range(5):
        learn()
    t_learn = (time.perf_counter() - t0) / 5
    t0 = time.perf_counter()
    for _ in range(5):
        with torch.no_grad():
            net(xa).argmax(1)
    t_act_row = (time.perf_counter() - t0) / 5 / n_act
    return 1e3 * t_learn, 1e3 * t_act_row


def cpu_baseline(snap, R, lay_tables, P, args, E):
    """Oracle (C restatement, OpenMP over envs) on the host cores, started from the GPU
    state of the first cpu_envs envs at the beginning of the warm-up steps (same episode
    phase), stepped with uniform random actions; plus the reference's learn/act in torch
    on the same cores, composed into the rate of the same full training step."""
    try:
        from oracle import oracle as orc
    except Exception as e:  # oracle not built: report, never fall back
        return {"error": f"oracle unavailable: {e}"}
    n = len(snap)
    olays = [orc.Layout.from_tables(t, P) for t in lay_tables]
    envs = []
    for st, li in snap:
        oe = orc.Env(olays[li], thmap=False)
        oe.load_state(st)
        envs.append((li, oe))
    threads = host_threads()
    steps = args.cpu_steps
    done_steps, dt = 0, 0.0
    for li, olay in enumerate(olays):  # per layout: run_batch steps envs of one layout
        group = [oe for (l, oe) in envs if l == li]
        if not group:
            continue
        acts = np.random.RandomState(li).randint(0, 5, size=(steps, len(group) * R)).astype(np.int32)
        t0 = time.perf_counter()
        k, _ = orc.run_batch(olay, group, steps, acts, nthreads=threads)
        dt += time.perf_counter() - t0
        done_steps += k
    env_rate = done_steps / dt
    out = {"value": env_rate, "unit": "env-steps/s", "cores": threads, "kind": "port",
           "nproc": os.cpu_count(), "cpu_model": cpu_model(),
           "sample": f"{n} envs x {steps} env.steps of the same workload from the GPU's state at the start of the "
                     f"warm-up steps (env.step only), OpenMP {threads} threads (all cores of this process's "
                     f"affinity set, capped by OMP_NUM_THREADS), {dt:.2f}s wall, {dt * threads:.1f} core-s; "
                     "compare with env_only_steps_per_s"}
    if args.mode == "train" and args.qnet == "mlp":
        t_learn, t_row = cpu_learner_ms(args, threads)
        t_step = E / env_rate * 1e3 + E * R * t_row + t_learn  # ms per full training step of E envs
        out["train_step"] = {"value": E / (t_step * 1e-3), "unit": "env-steps/s",
                             "learn_ms": t_learn, "act_us_per_row": 1e3 * t_row,
                             "what": "oracle env.step + torch-CPU act forward (E*R rows) + torch-CPU learn "
                                     f"(B={args.batch}, f32) on the same {threads} threads, composed per step "
                                     "of E envs; compare with value"}
    return out


if __name__ == "__main__":
    main()
