"""Independent Q-networks per agent in grouped launches.

Reference: Louvre_Evacuation/runners/train_double_dqn.py:35-56 trains one DQNAgent per robot
(each its own network, replay, dropout, clip_grad_norm_ and Adam); runners/train_qmix.py:39-118
trains one per agent under a MixingNetwork whose loss backpropagates into every agent. Here the
G networks (the MLP of DQNNetwork, 726-512-256-5, f32-accurate x3 operands) share every launch:
each kernel of the act and of the learn chain takes the net from its grid (evx_qmlp_*_g,
evx_td_loss_zero_g, include/evacx.h), and every per-net buffer -- flat parameters, gradients,
Adam moments, MFMA operand copies, activations -- is one slice of a [G][...] array.

* ``GroupedLearner.act``: robot g of env i (row i * G + g of the env's observation / action
  buffers) uses net g -- one launch for all robots of all envs.
* ``GroupedLearner.learn_obs``: net g learns on rows [g B, (g + 1) B) of the sampled batch
  (its own transitions): forward pair, TD loss, backward and clip + Adam, each one launch
  for all nets; per-net results equal G separate ``evacx.qnet.Learner`` steps bit for bit.
* ``GroupedQMix``: the QMIX learn step -- the agents' forwards, the mixer's loss and backward
  in one kernel (evx_qmix_loss: dQ of every agent at its taken action), the agents' grouped
  backward and per-agent clip + Adam, the mixer's clip_grad_norm_ + Adam.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional

import torch

from .env import _stream
from .qmlp import HID, HID2, K1X, NACT, MLPFast, _need, evx_qmlp_fwd_out, evx_qmlp_grads, mcheck, mlib
from .qnet import DROPOUT_P, FlatParams, evx_adam, layer_specs, param_shapes, qcheck, qlib


def _p(t):
    return None if t is None else t.data_ptr()


class GroupedMLP:
    """G MLPFast operand sets (x3) laid out as [G][...] arrays; ``c`` is net 0's evx_qmlp_params,
    which the grouped kernels advance per net."""

    def __init__(self, params: List[FlatParams], device):
        G = len(params)
        sizes = MLPFast.buffer_sizes(True)
        self.bufs = {k: torch.zeros(G, n, dtype=dt, device=device) for k, (n, dt) in sizes.items()}
        self.nets = [MLPFast(params[g], device, x3=True, store={k: v[g] for k, v in self.bufs.items()})
                     for g in range(G)]
        self.c = self.nets[0].c

    def repack(self):
        for n in self.nets:
            n.repack()


class GroupedLearner:
    """G independent DQN learners (MLP, x3 f32-accurate) stepping together."""

    def __init__(self, nets: int, device="cuda", lr=1e-4, gamma=0.99, max_norm=1.0, seed=0, betas=(0.9, 0.999),
                 eps=1e-8, init_seeds: Optional[List[int]] = None):
        if not 1 <= nets <= 64:
            raise ValueError("GroupedLearner: 1..64 nets")
        self.G, self.device = int(nets), torch.device(device)
        self.shapes = param_shapes(layer_specs("mlp"))
        self.npar = sum(int(torch.Size(s).numel()) for s in self.shapes.values())
        assert self.npar == int(mlib().evx_qmlp_nparams()), "MLP parameter count"
        f32 = dict(dtype=torch.float32, device=self.device)
        G = self.G
        self.flat = torch.zeros(G, self.npar, **f32)
        self.tflat = torch.zeros(G, self.npar, **f32)
        self.gflat = torch.zeros(G, self.npar, **f32)
        self.m = torch.zeros(G, self.npar, **f32)
        self.v = torch.zeros(G, self.npar, **f32)
        self.online = [FlatParams(self.shapes, self.device, data=self.flat[g]) for g in range(G)]
        self.target = [FlatParams(self.shapes, self.device, data=self.tflat[g]) for g in range(G)]
        self.grads = [FlatParams(self.shapes, self.device, data=self.gflat[g]) for g in range(G)]
        seeds = init_seeds if init_seeds is not None else [seed + g for g in range(G)]
        for g in range(G):
            self.online[g].init_like_torch(seeds[g])  # evacx.qnet.Learner(seed=seeds[g])'s initial weights
        self.tflat.copy_(self.flat)
        self.fast = GroupedMLP(self.online, self.device)
        self.fast_t = GroupedMLP(self.target, self.device)
        self.lr, self.gamma, self.max_norm, self.betas, self.eps = lr, gamma, max_norm, betas, eps
        self.seed, self.drop_stream, self.adam_step, self._act_calls = seed, 0, 0, 0
        self.drop_p = DROPOUT_P  # nn.Dropout(0.2) of DQNNetwork (0: off, tests)
        self.nss = int(mlib().evx_qmlp_norm_parts())
        self._ss = torch.zeros(G, self.nss, **f32)
        self.norm = torch.zeros(G, **f32)
        self.loss = torch.zeros(G, **f32)
        self._ws = {}

    def _buf(self, name, n, dtype):
        t = self._ws.get(name)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(n, dtype=dtype, device=self.device)
            self._ws[name] = t
        return t[:n]

    # ------------------------------------------------------------------ act
    def act(self, lay_c, obs: torch.Tensor, n: int, actions=None, q=None, epsilon=0.0, act_seed=0, act_offset=0,
            drop_p=DROPOUT_P, drop_seed=None, drop_stream=None):
        """DQNAgent.act of every agent: rows i * G + g of obs / q / actions (n rows per net) through
        net g (evx_qmlp_act_g); dropout active as in the reference's train-mode act."""
        G = self.G
        _need("act_g obs", obs, n * G, 8)
        _need("act_g q", q, n * G, NACT)
        _need("act_g actions", actions, n * G, 1)
        if drop_stream is None:  # a fresh mask stream per act call (above the learner's streams)
            self._act_calls += 1
            drop_stream = 0x40000000 + self._act_calls
        d = MLPFast._drop((self.seed if drop_seed is None else drop_seed, drop_stream, drop_p))
        o = evx_qmlp_fwd_out(q=_p(q), actions=_p(actions), epsilon=float(epsilon), act_seed=act_seed,
                             act_offset=act_offset)
        mcheck(mlib().evx_qmlp_act_g(C.byref(lay_c), obs.data_ptr(), n, G, C.byref(self.fast.c), C.byref(d),
                                     C.byref(o), _stream()), "qmlp_act_g")

    # ---------------------------------------------------------------- learn
    def learn_obs(self, lay_c, s_obs, a, r, done, s2_obs, B: int, update: bool = True):
        """One DQNAgent.learn step of every net: net g's batch is rows [g B, (g + 1) B) of s_obs /
        a / r / done / s2_obs. Returns the per-net losses [G] (device, no host sync)."""
        G = self.G
        if B <= 0 or B % 2:
            raise ValueError("learn_obs: B must be even and > 0")
        for name, t, w in (("s_obs", s_obs, 8), ("s2_obs", s2_obs, 8), ("a", a, 1), ("r", r, 1), ("done", done, 1)):
            _need("learn_obs " + name, t, G * B, w)
        X = self._buf("x", G * B * K1X, torch.int16)
        H1 = self._buf("h1", G * 2 * B * HID, torch.int16)
        H2 = self._buf("h2", G * B * HID2, torch.float32)
        Q = self._buf("q", G * B * NACT, torch.float32)
        H1t = self._buf("h1t", G * 2 * B * HID, torch.int16)
        Qt = self._buf("qt", G * B * NACT, torch.float32)
        self.drop_stream += 2
        d_on = MLPFast._drop((self.seed, self.drop_stream, self.drop_p))
        d_tg = MLPFast._drop((self.seed, self.drop_stream + 1, self.drop_p))
        o_on = MLPFast._out(H1, X, H2, Q)
        o_tg = MLPFast._out(H1t, None, None, Qt)
        mcheck(mlib().evx_qmlp_forward2_g(C.byref(lay_c), B, G, s_obs.data_ptr(), C.byref(self.fast.c), C.byref(d_on),
                                          C.byref(o_on), s2_obs.data_ptr(), C.byref(self.fast_t.c), C.byref(d_tg),
                                          C.byref(o_tg), _stream()), "qmlp_forward2_g")
        dQ = self._buf("dq", G * B * NACT, torch.float32)
        tw = self._buf("td_ws", max(1, int(qlib().evx_td_loss_ws_floats(B, G))), torch.float32)
        qcheck(qlib().evx_td_loss_zero_g(Q.data_ptr(), Qt.data_ptr(), NACT, a.data_ptr(), r.data_ptr(), done.data_ptr(),
                                         self.gamma, B, G, None, dQ.data_ptr(), self.loss.data_ptr(), None,
                                         self.gflat.data_ptr(), self.gflat.numel(), tw.data_ptr(), tw.numel(),
                                         _stream()), "td_loss_zero_g")
        self._backward(B, dQ, X, H1, H2)
        if update:
            self.step_optimizer()
        return self.loss

    def _backward(self, B, dQ, X, H1, H2):
        G = self.G
        dz2 = self._buf("dz2", G * 2 * B * HID2, torch.int16)
        dz1 = self._buf("dz1", G * 2 * B * HID, torch.int16)
        part = self._buf("part", G * int(mlib().evx_qmlp_backward_part_floats(B)), torch.float32)
        g0 = self.grads[0]
        g = evx_qmlp_grads(w1=g0["fc1.weight"].data_ptr(), b1=g0["fc1.bias"].data_ptr(), w2=g0["fc2.weight"].data_ptr(),
                           b2=g0["fc2.bias"].data_ptr(), w3=g0["fc3.weight"].data_ptr(), b3=g0["fc3.bias"].data_ptr(),
                           part=part.data_ptr())
        mcheck(mlib().evx_qmlp_backward_ss_g(C.byref(self.fast.c), B, G, dQ.data_ptr(), X.data_ptr(), H1.data_ptr(),
                                             H2.data_ptr(), float(self.drop_p), dz2.data_ptr(), dz1.data_ptr(),
                                             C.byref(g), self._ss.data_ptr(), _stream()), "qmlp_backward_ss_g")

    def step_optimizer(self):
        """clip_grad_norm_(net g, max_norm) + Adam for every net (one launch, evx_qmlp_adam_pack3_g)."""
        self.adam_step += 1
        h = evx_adam(lr=self.lr, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps, weight_decay=0.0,
                     step=self.adam_step)
        b = self.fast.bufs
        mcheck(mlib().evx_qmlp_adam_pack3_g(self.flat.data_ptr(), self.gflat.data_ptr(), self.m.data_ptr(),
                                            self.v.data_ptr(), float(self.max_norm or 0.0), C.byref(h),
                                            b["w1b"].data_ptr(), b["w1l"].data_ptr(), b["b1c"].data_ptr(),
                                            b["w2b"].data_ptr(), b["w2l"].data_ptr(), b["w2t"].data_ptr(),
                                            b["w2tl"].data_ptr(), b["w1o"].data_ptr(), b["w1ol"].data_ptr(),
                                            self._ss.data_ptr(), self.nss, self.norm.data_ptr(), self.G, _stream()),
               "qmlp_adam_pack3_g")

    def sync_target(self, nets: Optional[List[int]] = None):
        """agent.update_target_network() of the given nets (all by default)."""
        for g in (range(self.G) if nets is None else nets):
            self.tflat[g].copy_(self.flat[g])
            self.fast_t.nets[g].repack()

    def state_dict(self, g: int):
        """Net g's parameters in DQNNetwork's state_dict order (evacx.qnet.FlatParams)."""
        return self.online[g].state_dict()


class GroupedQMix:
    """QMIX learn step (runners/train_qmix.py:78-118) on a GroupedLearner of n agents: the agents'
    grouped forwards, evx_qmix_loss (both mixers, MSE, backward through the online mixer into every
    agent's dQ, the mixer's gradient), the grouped backward, per-agent clip_grad_norm_ + Adam and
    the mixer's clip_grad_norm_ + Adam (lr 1e-3)."""

    def __init__(self, agents: GroupedLearner, mix_lr: float = 1e-3, embed: int = 32, seed: int = 0,
                 mixing: Optional[torch.nn.Module] = None):
        self.A = agents
        n = agents.G
        if embed != 32:
            raise ValueError("GroupedQMix: embed_dim 32 (the reference's MixingNetwork)")
        self.nmix = int(mlib().evx_qmix_nparams(n))
        f32 = dict(dtype=torch.float32, device=agents.device)
        self.mix = torch.zeros(self.nmix, **f32)
        if mixing is not None:  # a MixingNetwork (evacx.qmix / the reference's): its state_dict order
            self.mix.copy_(torch.cat([p.detach().reshape(-1).float() for p in mixing.state_dict().values()]))
        else:  # MixingNetwork.__init__: fc1_weight, fc2_weight ~ randn, biases zero
            g = torch.Generator().manual_seed(seed)
            w1 = torch.randn(n, embed, generator=g)
            w2 = torch.randn(embed, 1, generator=g)
            self.mix.copy_(torch.cat([w1.reshape(-1), torch.zeros(embed), w2.reshape(-1), torch.zeros(1)]))
        self.mix_t = self.mix.clone()
        self.mix_g = torch.zeros_like(self.mix)
        self.mix_m = torch.zeros_like(self.mix)
        self.mix_v = torch.zeros_like(self.mix)
        self.mix_step = 0
        self.mix_lr = mix_lr
        self.loss = torch.zeros(1, **f32)
        self.mix_norm = torch.zeros(1, **f32)
        self._scratch = torch.zeros(2048, **f32)

    def __call__(self, lay_c, s_obs, a, r, done, s2_obs, B: int):
        """s_obs / s2_obs [n][B] compact observations, a [n][B] int32 (agent-major), r / done [B] (the
        joint reward and done flag). Returns the loss tensor [1] (device)."""
        A, n = self.A, self.A.G
        X = A._buf("x", n * B * K1X, torch.int16)
        H1 = A._buf("h1", n * 2 * B * HID, torch.int16)
        H2 = A._buf("h2", n * B * HID2, torch.float32)
        Q = A._buf("q", n * B * NACT, torch.float32)
        H1t = A._buf("h1t", n * 2 * B * HID, torch.int16)
        Qt = A._buf("qt", n * B * NACT, torch.float32)
        for name, t, w in (("s_obs", s_obs, 8), ("s2_obs", s2_obs, 8), ("a", a, 1)):
            _need("qmix " + name, t, n * B, w)
        _need("qmix r", r, B, 1)
        _need("qmix done", done, B, 1)
        A.drop_stream += 2
        d_on = MLPFast._drop((A.seed, A.drop_stream, A.drop_p))
        d_tg = MLPFast._drop((A.seed, A.drop_stream + 1, A.drop_p))
        o_on = MLPFast._out(H1, X, H2, Q)
        o_tg = MLPFast._out(H1t, None, None, Qt)
        mcheck(mlib().evx_qmlp_forward2_g(C.byref(lay_c), B, n, s_obs.data_ptr(), C.byref(A.fast.c), C.byref(d_on),
                                          C.byref(o_on), s2_obs.data_ptr(), C.byref(A.fast_t.c), C.byref(d_tg),
                                          C.byref(o_tg), _stream()), "qmlp_forward2_g")
        dQ = A._buf("dq", n * B * NACT, torch.float32)
        part = A._buf("mixpart", int(mlib().evx_qmix_part_floats(B, n)), torch.float32)
        rc = mlib().evx_qmix_loss(Q.data_ptr(), Qt.data_ptr(), NACT, a.data_ptr(), r.data_ptr(), done.data_ptr(),
                                  A.gamma, B, n, self.mix.data_ptr(), self.mix_t.data_ptr(), dQ.data_ptr(),
                                  self.mix_g.data_ptr(), self.loss.data_ptr(), part.data_ptr(), A.gflat.data_ptr(),
                                  A.gflat.numel(), _stream())
        if rc != 0:
            raise RuntimeError(f"qmix_loss failed ({rc}): {mlib().evx_qmix_last_error().decode()}")
        A._backward(B, dQ, X, H1, H2)
        A.step_optimizer()  # clip_grad_norm_(agent_i, 1.0) + agent_i.optimizer.step()
        L = qlib()
        qcheck(L.evx_sumsq_norm(self.mix_g.data_ptr(), self.nmix, self._scratch.data_ptr(), self._scratch.numel(),
                                self.mix_norm.data_ptr(), _stream()), "sumsq_norm")
        self.mix_step += 1
        h = evx_adam(lr=self.mix_lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=self.mix_step)
        qcheck(L.evx_clip_adam(self.mix.data_ptr(), self.mix_g.data_ptr(), self.mix_m.data_ptr(), self.mix_v.data_ptr(),
                               self.nmix, self.mix_norm.data_ptr(), float(A.max_norm or 0.0), C.byref(h), _stream()),
               "clip_adam")
        return self.loss

    def sync_targets(self):
        """agent.update_target_network() for every agent + target_mixing <- mixing (:116-118)."""
        self.A.sync_target()
        self.mix_t.copy_(self.mix)
