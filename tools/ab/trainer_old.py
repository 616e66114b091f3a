"""Vectorised multi-agent DQN training loop, fully device-resident.

One ``step()`` = for all E envs x R robots of this rank:
  act      -- expand the compact observations, Q-forward (dropout active, as the
              reference's act never leaves train mode), epsilon-greedy (evx_act)
  env.step -- evx_env_step (the CA, bit-exact with the reference's step)
  push     -- E*R transitions into the replay ring (team reward/done per env)
  learn    -- sample B, online + target forwards, TD loss, backward, optional
              gradient all-reduce (RCCL over xGMI when world > 1), clip + Adam
  reset    -- auto-reset of finished envs (reference reset semantics) fused into
              the env.step launch; the heavy-first dispatch order of the next
              env.step and the next act's env order (evx_env_orders) follow it in
              one launch on the same stream
With groups > 1 the envs are split into parts that run act -> env.step -> push on
their own streams, so one part's env.step tail overlaps the others' work.

Reference: runners/train_double_dqn.py:43-69 (independent robots, shared team
reward) generalised to R robots and E envs; DQNAgent.act/remember/learn
(agents/dqn_agent.py:97-168). No host syncs inside ``step()``.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional

import numpy as np
import torch

from . import _lib
from ._lib import evx_replay
from .env import OBS_WORDS, DeviceLayout, VecEnv, _ptr, _stream
from .qmlp import act_ws_ints
from .qnet import DROPOUT_P, Learner, qcheck, qlib


class Replay:
    """Uniform replay ring of compact observations in HBM."""

    def __init__(self, capacity: int, device):
        self.capacity = int(capacity)
        i32 = dict(dtype=torch.int32, device=device)
        self.s = torch.zeros(self.capacity * OBS_WORDS, **i32)
        self.s2 = torch.zeros(self.capacity * OBS_WORDS, **i32)
        self.a = torch.zeros(self.capacity, **i32)
        self.r = torch.zeros(self.capacity, dtype=torch.float32, device=device)
        self.done = torch.zeros(self.capacity, dtype=torch.uint8, device=device)
        self.c = evx_replay(capacity=self.capacity, s=self.s.data_ptr(), s2=self.s2.data_ptr(), a=self.a.data_ptr(),
                            r=self.r.data_ptr(), done=self.done.data_ptr())
        self.pos = 0
        self.size = 0

    def push(self, s, s2, a, r_env, done_env, n, agents_per_env, s2_term=None):
        """s2_term: terminal observations of auto-reset envs (taken where done_env)."""
        L = _lib.lib()
        if s2_term is None:
            L.evx_replay_push.argtypes = [C.POINTER(evx_replay), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_void_p]
            qcheck(L.evx_replay_push(C.byref(self.c), s.data_ptr(), s2.data_ptr(), a.data_ptr(), r_env.data_ptr(),
                                     done_env.data_ptr(), n, agents_per_env, self.pos, _stream()), "replay_push")
        else:
            L.evx_replay_push_term.argtypes = [C.POINTER(evx_replay)] + [C.c_void_p] * 6 + [C.c_int32, C.c_int32,
                                                                                          C.c_int64, C.c_void_p]
            qcheck(L.evx_replay_push_term(C.byref(self.c), s.data_ptr(), s2.data_ptr(), s2_term.data_ptr(),
                                          a.data_ptr(), r_env.data_ptr(), done_env.data_ptr(), n, agents_per_env,
                                          self.pos, _stream()), "replay_push_term")
        self.pos = (self.pos + n) % self.capacity
        self.size = min(self.capacity, self.size + n)

    def push_orders(self, env, perm, s, s2, a, r_env, done_env, n, agents_per_env, s2_term=None, sample=None):
        """push with env's next dispatch order and act env order (perm) in the same launch
        (evx_env_orders_push_sample; power-of-two capacity). sample = (B, seed, offset, out): also
        draw the learn step's batch into out, as sample() would right after the push."""
        size = min(self.capacity, self.size + n)
        B, seed, offset, out = sample if sample is not None else (0, 0, 0, None)
        o = (lambda k: out[k].data_ptr()) if out is not None else (lambda k: None)
        qcheck(_lib.lib().evx_env_orders_push_sample(
            C.byref(env.lay.c), C.byref(env.c), _ptr(perm), C.byref(self.c), s.data_ptr(), s2.data_ptr(),
            _ptr(s2_term), a.data_ptr(), r_env.data_ptr(), done_env.data_ptr(), n, agents_per_env, self.pos,
            B, size, seed, offset, o("s"), o("s2"), o("a"), o("r"), o("done"), _stream()), "env_orders_push_sample")
        self.pos = (self.pos + n) % self.capacity
        self.size = size

    def window(self, n_next):
        """(base, count): the entries already in the ring that a push of n_next
        transitions does not overwrite -- the newest min(size, capacity - n_next)."""
        count = min(self.size, self.capacity - n_next)
        return (self.pos - count) % self.capacity, count

    def sample_window(self, base, count, B, seed, offset, out):
        L = _lib.lib()
        L.evx_replay_sample_window.argtypes = [C.POINTER(evx_replay), C.c_int64, C.c_int64, C.c_int32, C.c_uint64,
                                               C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_void_p]
        qcheck(L.evx_replay_sample_window(C.byref(self.c), base, count, B, seed, offset, out["s"].data_ptr(),
                                          out["s2"].data_ptr(), out["a"].data_ptr(), out["r"].data_ptr(),
                                          out["done"].data_ptr(), None, _stream()), "replay_sample_window")

    def sample(self, B, seed, offset, out):
        L = _lib.lib()
        L.evx_replay_sample.argtypes = [C.POINTER(evx_replay), C.c_int64, C.c_int32, C.c_uint64, C.c_uint64,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p]
        qcheck(L.evx_replay_sample(C.byref(self.c), self.size, B, seed, offset, out["s"].data_ptr(),
                                   out["s2"].data_ptr(), out["a"].data_ptr(), out["r"].data_ptr(),
                                   out["done"].data_ptr(), None, _stream()), "replay_sample")


class _Group:
    """One part of the envs with its own stream chain (act -> env.step -> push): with
    several groups, one group's env.step launch tail (its heaviest envs, few waves)
    overlaps the other groups' act and env.step instead of idling the chip."""

    def __init__(self, env: VecEnv, g: int, row0: int, actions: torch.Tensor, device):
        self.env, self.g, self.row0 = env, g, row0
        self.n = env.E * env.lay.R
        self.actions = actions  # this group's rows of the trainer's action buffer
        # act, env.step, push on a high-priority stream: the learn stream's workgroups
        # then fill the env launch's tail instead of competing for its first slots
        self.main = torch.cuda.Stream(device=device, priority=-1)
        # one group: the next step's orders (evx_env_orders) beside the learn; extra resets
        self.side = torch.cuda.Stream(device=device, priority=0)
        cur = torch.cuda.current_stream(device)
        self.ev_push = torch.cuda.Event()
        self.ev_push.record(cur)
        self.ev_act = torch.cuda.Event()
        self.ev_order = torch.cuda.Event()
        self.ev_order.record(cur)
        self.perm = None  # the act's env order over this group's envs (x3 table path), or None
        self.act_ws = None  # the x3 act's workspace (evx_qmlp_fwd_out.act_ws), made at the first act


class VecTrainer:
    def __init__(self, layout: DeviceLayout, E: int, seed_base: int = 1234, env_offset: int = 0,
                 kind: str = "mlp", precision: str = "f32", batch: int = 4096, replay_capacity: int = 1 << 20,
                 lr: float = 1e-4, gamma: float = 0.99, epsilon: float = 1.0, epsilon_min: float = 0.02,
                 epsilon_decay: float = 0.9995, target_every: int = 1000, learner_seed: int = 0,
                 grad_hook=None, learn_every: int = 1, lagged_learn: bool = False, replay: str = "uniform",
                 prio_alpha: float = 0.6, prio_beta0: float = 0.4, prio_beta_steps: int = 100000,
                 prio_eps: float = 1e-6, groups: int = 1, layout_of=None, world_envs: Optional[int] = None,
                 nets: str = "shared", act_table: Optional[bool] = None):
        """groups: the envs are split into this many parts, each stepping on its own
        stream chain (see _Group), group g's act after group g - 1's (it overlaps that
        group's env.step); neither the env results nor the act's dropout masks (one stream
        per step, rows keyed by global agent id) depend on it.
        layout: a DeviceLayout, or an evacx.env.LayoutSet with layout_of = each env's
        layout (per-env layouts; observations in the replay carry their layout).
        world_envs: envs over all ranks (default E). This rank's envs are global ids
        env_offset .. env_offset + E - 1; the act's epsilon draws and dropout rows are keyed
        by global agent id, so every env's trajectory is the same at any GPU count as long
        as the actions do not depend on the (rank-shared) weights' history.
        nets: "shared" (one Q-network for every robot) or "per_robot" (robot r of every env has
        its own network, memory and optimizer, as runners/train_double_dqn.py:35-56 gives each
        robot its own DQNAgent: evacx.qgroup.GroupedLearner, batch / R transitions per net per
        learn step, strict schedule, one GPU) or "qmix" (per-robot nets under a QMIX mixer,
        runners/train_qmix.py: batch / R joint env-steps per learn step, evacx.qgroup.GroupedQMix)."""
        if precision not in ("f32", "bf16", "exact"):
            raise ValueError(f"precision must be 'f32', 'bf16' or 'exact', not {precision!r}")
        self.lay, self.E, self.R = layout, E, layout.R
        self.device = layout.device
        # the push reads env.obs_prev: no copy per step
        self.env = VecEnv(layout, E, obs_buffers=2, layout_of=layout_of)
        self.env.seed([seed_base + env_offset + i for i in range(E)])
        self.env.reset()
        parts = self.env.split(groups) if groups > 1 else [self.env]
        self.per_robot = nets in ("per_robot", "qmix")
        if nets not in ("shared", "per_robot", "qmix"):
            raise ValueError(f"nets must be 'shared', 'per_robot' or 'qmix', not {nets!r}")
        if self.per_robot:
            if kind != "mlp" or precision != "f32" or groups != 1 or lagged_learn or replay != "uniform" or \
                    layout_of is not None or grad_hook is not None:
                raise ValueError("per_robot nets: MLP, f32, one group, strict schedule, uniform replay, one layout, "
                                 "one GPU")
            if batch % (2 * self.R) or replay_capacity % self.R:
                raise ValueError("per_robot nets: batch a multiple of 2 R, replay capacity a multiple of R")
            from .qgroup import GroupedLearner, GroupedQMix
            self.glearner = GroupedLearner(self.R, self.device, lr=lr, gamma=gamma, seed=learner_seed)
            # qmix: the R robots of an env are the agents of runners/train_qmix.py -- joint samples
            # (the same env-steps for every agent), the mixer's loss over the team reward
            self.qmix = GroupedQMix(self.glearner, seed=learner_seed) if nets == "qmix" else None
        # precision: "f32" -- f32-accurate x3 (the fused MLP kernels; the conv net's implicit-GEMM
        # convolutions, bf16 hi/lo operand pairs); "bf16"; "exact" -- every product on the exact-f32
        # MFMA GEMMs (evx_gemm f32, no fused kernels: the golden-test path, either kind)
        lprec = "x3" if (kind == "conv" and precision == "f32") else precision
        self.learner = Learner(kind=kind, device=self.device, lr=lr, gamma=gamma, precision=lprec,
                               seed=learner_seed) if not self.per_robot else None
        # the arithmetic the Q-network actually runs: "x3" (f32 operands as bf16 hi + lo pairs on the
        # bf16 MFMA, f32 accumulation: f32 within the tests' stated tolerances), "f32" (exact f32
        # MFMA) or "bf16" -- read from what the learner built
        if self.per_robot:
            self.q_arith = "x3"
        elif self.learner.fast is not None:
            self.q_arith = "x3" if self.learner.fast.x3 else "bf16"
        else:
            self.q_arith = {"exact": "f32"}.get(lprec, lprec)
        if self.learner is not None:
            self.learner.grad_hook = grad_hook
        # replay: "uniform" (DQNAgent.memory's random.sample) or "prioritized" (evacx.prio:
        # device sum/min trees, importance-weighted loss, beta annealed to 1)
        self.prio = replay == "prioritized"
        if self.prio:
            from .prio import PrioReplay
            self.replay = PrioReplay(replay_capacity, self.device, alpha=prio_alpha, eps=prio_eps)
        elif replay == "uniform":
            self.replay = Replay(replay_capacity, self.device)
        else:
            raise ValueError(f"replay must be 'uniform' or 'prioritized', not {replay!r}")
        self.prio_beta0, self.prio_beta_steps = prio_beta0, prio_beta_steps
        self.batch = batch
        self.epsilon, self.epsilon_min, self.epsilon_decay = epsilon, epsilon_min, epsilon_decay
        self.target_every, self.learn_every = target_every, learn_every
        # lagged_learn: learn step t samples the transitions pushed up to step t-1 and runs
        # on its own stream concurrently with env.step t (see step())
        self.lagged = lagged_learn
        n = E * self.R
        self.n_agents = n
        self.agent0 = env_offset * self.R  # global agent id of this rank's first robot
        self.n_world = (E if world_envs is None else int(world_envs)) * self.R
        if self.agent0 % 2:
            raise ValueError("env_offset * R must be even (dropout hash rows come in pairs)")
        self.actions = torch.zeros(n, dtype=torch.int32, device=self.device)
        ng = n // len(parts)
        self.groups: List[_Group] = [_Group(p, g, g * ng, self.actions[g * ng:(g + 1) * ng], self.device)
                                     for g, p in enumerate(parts)]
        self.main = self.groups[0].main
        self.samp = dict(s=torch.zeros(batch * OBS_WORDS, dtype=torch.int32, device=self.device),
                         s2=torch.zeros(batch * OBS_WORDS, dtype=torch.int32, device=self.device),
                         a=torch.zeros(batch, dtype=torch.int32, device=self.device),
                         r=torch.zeros(batch, dtype=torch.float32, device=self.device),
                         done=torch.zeros(batch, dtype=torch.uint8, device=self.device))
        if self.prio:
            self.samp.update(idx=torch.zeros(batch, dtype=torch.int64, device=self.device),
                             w=torch.zeros(batch, dtype=torch.float32, device=self.device),
                             td=torch.zeros(batch, dtype=torch.float32, device=self.device))
        # replay sampling: per rank (each rank samples its own shard); act draws: one key for
        # all ranks (counters are global agent ids)
        self.seed = learner_seed * 7919 + env_offset + 17
        self.act_seed = learner_seed * 7919 + 17
        self.t = 0
        self.learn_steps = 0
        cur = torch.cuda.current_stream(self.device)
        self.ev_reset = torch.cuda.Event()
        self.ev_reset.record(cur)
        self.reset_pending = False
        self.join_caller = True  # the first step waits for the caller's stream (set-up work)
        self._orders_side = False  # the last step's orders were made on the side stream (act waits for them)
        self._presampled = False   # this step's learn batch was drawn by the push launch
        self.lstream = torch.cuda.Stream(device=self.device, priority=0)
        self.ev_learned = torch.cuda.Event()
        self.ev_learned.record(cur)
        self.last_loss: Optional[torch.Tensor] = None
        # bf16 MLP: act and learn straight from compact observations (csrc/qmlp.hip)
        self.fast = self.learner.fast if self.learner is not None else None
        if self.fast is None:
            self.lagged = False  # the lagged schedule's two-phase learn needs the fused MLP path
        self._perm = None
        if act_table is None:
            act_table = True
        if self.fast is not None and self.fast.x3 and layout_of is None and act_table:
            # act fast path: envs past the fire's last step start fc1 from a per-centre table of the
            # static features' contribution (rebuilt with every weight update) and add only the
            # occupancy columns; the act visits those envs first (VecEnv.act_perm) so its row tiles
            # are uniform. x3 only (the table replaces ~3/4 of fc1's products); bf16: off (the
            # rebuild costs what the act saves, tools/gpu_ab_static.sh)
            lc = self.lay.c  # centres only where robots can be (Map.robot_range): 55 of 130 columns at cfg3
            xr = (max(lc.rx_lo, 0), min(lc.rx_hi, lc.L + 1))
            self.fast.attach_static(lc, lc.L, lc.W, lc.t_max, x_range=xr)
            # the target net's table too (rebuilt at each target sync): the learner's target
            # forward (the fused act kernel at B >= 32768) starts fc1 from it for replay rows
            # past the fire's last step
            self.learner.fast_t.attach_static(lc, lc.L, lc.W, lc.t_max, x_range=xr)
            # the act's env order, per group (each group's act visits its own envs)
            self._perm = torch.zeros(E, dtype=torch.int32, device=self.device)
            for grp in self.groups:
                grp.perm = self._perm[grp.g * grp.env.E:(grp.g + 1) * grp.env.E]
        for grp in self.groups:  # the first step's orders (the reset wrote every class byte)
            grp.env.compute_orders(perm=grp.perm)

    def _act(self, grp: _Group):
        """DQNAgent.act in train mode for one group's robots: dropout active, epsilon-greedy
        over argmax Q; the epsilon draws are counted over all E*R robots of the step."""
        g0 = self.agent0 + grp.row0  # global agent id of the group's first robot
        off = self.t * self.n_world + g0
        if self.per_robot:  # robot r of every env through net r, one launch
            self.glearner.act(self.lay.c, grp.env.obs, grp.env.E, actions=grp.actions, epsilon=float(self.epsilon),
                              act_seed=self.act_seed, act_offset=off)
            return
        if self.fast is not None:  # one mask stream per step (act_streams), rows keyed by global agent id
            if grp.act_ws is None and act_ws_ints(grp.n) > 0:  # the persistent act's list of tiles off the table path
                grp.act_ws = torch.zeros(act_ws_ints(grp.n), dtype=torch.int32, device=self.device)
            self.fast.act(self.lay.c, grp.env.obs, grp.n,
                          drop=(self.learner.seed, self.learner.drop_stream, DROPOUT_P, None, g0),
                          actions=grp.actions, epsilon=float(self.epsilon), act_seed=self.act_seed, act_offset=off,
                          perm=grp.perm, rows_per_env=0 if grp.perm is None else self.R, ws=grp.act_ws)
            return
        x = grp.env.expand_obs(torch.float32)  # [E/G, R, 11, 11, 6]
        # per-group scratch: the groups' acts run concurrently on their own streams
        Q = self.learner.q_values(x.view(grp.n, 11, 11, 6), train=True, tag=f"act{grp.g}" if grp.g else "act")
        qcheck(qlib().evx_act(Q.data_ptr(), grp.n, self.learner.actions, float(self.epsilon), self.act_seed, off,
                              grp.actions.data_ptr(), _stream()), "act")

    def _act_stream(self):
        """A fresh dropout mask stream for this step's act: every group's act draws from it (rows keyed
        by global agent id), so the masks do not depend on the group count."""
        if self.fast is not None and not self.per_robot:
            self.learner.drop_stream += 1

    def act(self):
        """Launch DQNAgent.act for every robot of every env on the trainer's stream and return
        the actions buffer. The kernels run asynchronously: read the returned tensor only after
        sync() (or on a stream that waits for the trainer's), since the next step overwrites it."""
        self._act_stream()
        for grp in self.groups:
            self._act(grp)
        return self.actions

    def learn(self, window=None, phase: str = "all"):
        """window: (base, count) of the replay ring to sample from (default: all of it).
        phase: "all", or "grads" (sample .. backward) then "update" (clip+Adam, bf16
        repack, epsilon, target sync) -- the update may wait for readers of the weights."""
        if self.per_robot:  # every robot's net on batch / R of its own transitions
            Bn = self.batch // self.R
            if self.replay.size < self.batch:
                return None
            L = _lib.lib()
            L.evx_replay_sample_agents.argtypes = [C.POINTER(evx_replay), C.c_int64, C.c_int32, C.c_int32, C.c_uint64,
                                                   C.c_uint64] + [C.c_void_p] * 6
            sp = self.samp
            fn = L.evx_replay_sample_joint if self.qmix is not None else L.evx_replay_sample_agents
            fn.argtypes = L.evx_replay_sample_agents.argtypes
            qcheck(fn(C.byref(self.replay.c), self.replay.size, Bn, self.R, self.seed + 1, self.learn_steps * self.batch,
                      sp["s"].data_ptr(), sp["s2"].data_ptr(), sp["a"].data_ptr(), sp["r"].data_ptr(),
                      sp["done"].data_ptr(), _stream()), "replay_sample_agents/joint")
            if self.qmix is not None:  # agent 0's rows carry the team reward / done of the sampled env-steps
                loss = self.qmix(self.lay.c, sp["s"], sp["a"], sp["r"], sp["done"], sp["s2"], Bn)
            else:
                loss = self.glearner.learn_obs(self.lay.c, sp["s"], sp["a"], sp["r"], sp["done"], sp["s2"], Bn)
            self.learn_steps += 1
            if self.epsilon > self.epsilon_min:
                self.epsilon *= self.epsilon_decay
            if self.learn_steps % self.target_every == 0:
                if self.qmix is not None:
                    self.qmix.sync_targets()
                else:
                    self.glearner.sync_target()
            return loss
        if phase != "update":
            if (self.replay.size if window is None else window[1]) < self.batch:
                return None
            w = td = None
            if self.prio:
                # the trees only hold exposed slots: the window is implicit (hidden slots have 0 mass)
                beta = min(1.0, self.prio_beta0 + (1.0 - self.prio_beta0) * self.learn_steps / self.prio_beta_steps)
                w, td = self.samp["w"], self.samp["td"]
                self.replay.sample_prio(self.batch, beta, self.seed + 1, self.learn_steps * self.batch, self.samp,
                                        self.samp["idx"], w)
            elif window is None:
                if not self._presampled:  # (drawn by the push launch of this step)
                    self.replay.sample(self.batch, self.seed + 1, self.learn_steps * self.batch, self.samp)
                self._presampled = False
            else:
                self.replay.sample_window(window[0], window[1], self.batch, self.seed + 1,
                                          self.learn_steps * self.batch, self.samp)
            if self.fast is not None:
                loss = self.learner.learn_obs(self.lay.c, self.samp["s"], self.samp["a"], self.samp["r"],
                                              self.samp["done"], self.samp["s2"], self.batch, update=phase == "all",
                                              weights=w, td_abs=td)
            else:
                assert phase == "all", "a two-phase learn needs the fused MLP path"
                s = self.env.expand_obs(torch.float32, self.samp["s"]).view(self.batch, 11, 11, 6)
                s2 = self.env.expand_obs(torch.float32, self.samp["s2"]).view(self.batch, 11, 11, 6)
                loss = self.learner.learn(s, self.samp["a"], self.samp["r"], self.samp["done"], s2, weights=w,
                                          td_abs=td)
            if self.prio:
                self.replay.update(self.samp["idx"], td, self.batch)
            if phase == "grads":
                return loss
        else:
            self.learner.step_optimizer()
            loss = self.learner.loss
        self.learn_steps += 1
        if self.epsilon > self.epsilon_min:  # DQNAgent.learn epsilon schedule (agents/dqn_agent.py:163-164)
            self.epsilon *= self.epsilon_decay
        if self.learn_steps % self.target_every == 0:
            self.learner.sync_target()
        return loss

    def step(self, extra_reset: Optional[torch.Tensor] = None, ev_env=None, ev_learn=None, ev_act=None):
        """One training step. Finished envs are reset inside the env.step launch
        (auto-reset: the reset of an env that ends runs in its own wave, in the shadow
        of the launch's heavy envs); the replay push takes their terminal observations.
        The heavy-first dispatch order of each group's next env.step and the next act's
        env order come from one launch over the class bytes the step wrote
        (evx_env_orders): one group on its side stream beside the push and the learn (the
        act waits for it, long complete by then), several groups on their own streams.
        extra_reset: bool [E] of further envs to reset (benchmark staggering, side
        stream); ev_env / ev_learn:
        optional (start, end) CUDA events (env: group 0's env.step); ev_act: group 0's act.

        Default order is the reference's (act, env.step, remember, learn). With
        lagged_learn the learn step runs on its own stream from the ring as it was
        before this step's push (minus the slots the push overwrites): its gradients
        overlap act and env.step, its weight update waits for every group's act to have
        read the weights, and the next acts wait for the update."""
        caller = torch.cuda.current_stream(self.device)
        join = self.join_caller
        if self.join_caller or extra_reset is not None:  # inputs made on the caller's stream
            for grp in self.groups:
                grp.main.wait_stream(caller)
            self.join_caller = False
        G = self.groups
        # one group, uniform replay, no warm-up reset: the push and the next step's orders in one launch
        # on the main stream (no side-stream event); otherwise the orders on the side stream
        fused = (len(G) == 1 and extra_reset is None and type(self.replay) is Replay
                 and (self.replay.capacity & (self.replay.capacity - 1)) == 0)
        reset_wait, self.reset_pending = self.reset_pending, False
        self._presampled = False
        self._act_stream()
        # act: every group on its own stream, after the previous update (lagged) or learn
        for grp in G:
            with torch.cuda.stream(grp.main):
                if reset_wait:  # a cross-stream wait costs a gap: only when there was a reset
                    grp.main.wait_event(self.ev_reset)
                if self.lagged or grp.g > 0:
                    grp.main.wait_event(self.ev_learned)
                if grp.g > 0:  # the acts run one after the other: act g overlaps env.step g - 1
                    grp.main.wait_event(G[grp.g - 1].ev_act)
                if len(G) == 1 and self._orders_side:  # the orders from the side stream
                    grp.main.wait_event(grp.ev_order)
                if ev_act is not None and grp.g == 0:
                    ev_act[0].record(grp.main)
                self._act(grp)
                if ev_act is not None and grp.g == 0:
                    ev_act[1].record(grp.main)
                if self.lagged or grp.g + 1 < len(G):  # read by the update / the next group's act
                    grp.ev_act.record(grp.main)
        if self.lagged:
            # learn t: gradients from the ring as it stood after push t-1 (minus the slots
            # push t overwrites), overlapping act t and env.step t; the weight update
            # waits until every act t has read the weights, and act t+1 waits for it
            win = self.replay.window(self.n_agents)
            do_learn = self.t % self.learn_every == 0 and win[1] >= self.batch and self.fast is not None
            with torch.cuda.stream(self.lstream):
                for grp in G:
                    self.lstream.wait_event(grp.ev_push)
                if ev_learn is not None:
                    ev_learn[0].record(self.lstream)
                if self.prio:  # push t-1 visible, the slots push t overwrites hidden
                    self.replay.expose(n_hide=self.n_agents)
                if do_learn:
                    self.learn(window=win, phase="grads")
                for grp in G:
                    self.lstream.wait_event(grp.ev_act)
                self.last_loss = self.learn(phase="update") if do_learn else None
                if ev_learn is not None:
                    ev_learn[1].record(self.lstream)
                self.ev_learned.record(self.lstream)
        # a cross-stream reader of the push: the lagged learn stream, group 0's learn, a reset
        for grp in G:
            with torch.cuda.stream(grp.main):
                if ev_env is not None and grp.g == 0:
                    ev_env[0].record(grp.main)
                grp.env.step(grp.actions, order=False, auto_reset=True)
                if ev_env is not None and grp.g == 0:
                    ev_env[1].record(grp.main)
                if fused:
                    # the strict schedule's learn batch drawn in the same launch (the ring after this push)
                    smp = None
                    if (not self.lagged and not self.prio and not self.per_robot and self.t % self.learn_every == 0
                            and min(self.replay.capacity, self.replay.size + grp.n) >= self.batch):
                        smp = (self.batch, self.seed + 1, self.learn_steps * self.batch, self.samp)
                    self.replay.push_orders(grp.env, grp.perm, grp.env.obs_prev, grp.env.obs, grp.actions,
                                            grp.env.reward, grp.env.done, grp.n, self.R, s2_term=grp.env.obs_term,
                                            sample=smp)
                    self._presampled = smp is not None
                else:
                    self.replay.push(grp.env.obs_prev, grp.env.obs, grp.actions, grp.env.reward, grp.env.done,
                                     grp.n, self.R, s2_term=grp.env.obs_term)
                if len(G) > 1:  # several groups: the orders on this stream, after the push
                    grp.env.compute_orders(perm=grp.perm)
                if not fused or self.lagged:  # read by the side stream / the lagged learn stream
                    grp.ev_push.record(grp.main)
        if extra_reset is not None:  # after every group's push, on group 0's side stream (warm-up only)
            side = G[0].side
            extra_reset.record_stream(side)  # the caller may free it before the side stream reads it
            with torch.cuda.stream(side):
                side.wait_stream(caller)
                for grp in G:
                    side.wait_event(grp.ev_push)
                self.env.reset(mask=extra_reset & ~self.env.done.bool())
                if len(G) > 1:
                    for grp in G:  # the orders again, with the reset envs' new classes
                        grp.env.compute_orders(perm=grp.perm)
                self.ev_reset.record(side)
            self.reset_pending = True
        self._orders_side = len(G) == 1 and not fused
        if self._orders_side:
            # the next step's dispatch order and the next act's env order from the class bytes the
            # step (and a reset) just wrote, auto-reset envs included: one launch on the side stream,
            # beside the learn's first kernels
            grp = G[0]
            with torch.cuda.stream(grp.side):
                grp.side.wait_event(grp.ev_push)  # (after an extra reset: the same stream)
                grp.env.compute_orders(perm=grp.perm)
                grp.ev_order.record(grp.side)
        if not self.lagged:  # the reference's order: learn after every group's push, on group 0's stream
            m = G[0].main
            with torch.cuda.stream(m):
                for grp in G[1:]:
                    m.wait_event(grp.ev_push)
                if self.prio:
                    self.replay.expose()
                if ev_learn is not None:
                    ev_learn[0].record(m)
                if self.t % self.learn_every == 0:
                    self.last_loss = self.learn()
                if ev_learn is not None:
                    ev_learn[1].record(m)
                if len(G) > 1:
                    self.ev_learned.record(m)
        self._presampled = False
        self.t += 1

    def sync(self):
        """Make the current stream wait for all work of the steps so far. step() runs on
        the trainer's own streams and does not join the caller's stream each step (a
        cross-stream round trip costs tens of microseconds); read results after sync()."""
        cur = torch.cuda.current_stream(self.device)
        for grp in self.groups:
            cur.wait_stream(grp.main)
            cur.wait_event(grp.ev_order)
        cur.wait_event(self.ev_reset)
        cur.wait_event(self.ev_learned)
        self.join_caller = True


def make_allreduce_hook(dist, world: int):
    """Average the flat gradient buffer over ranks (one collective per learn step)."""
    backend = dist.get_backend()

    def hook(flat):
        if backend == "nccl":
            dist.all_reduce(flat, op=dist.ReduceOp.AVG)
        else:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM)
            flat.div_(world)
    return hook
