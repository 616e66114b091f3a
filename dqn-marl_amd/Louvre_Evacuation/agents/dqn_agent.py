"""Drop-in ``DQNNetwork`` / ``DQNAgent`` backed by the HIP learner kernels.

Mirrors the reference's agents/dqn_agent.py: constructor and hyper-parameters
(:67-95), ``remember`` (:97-99), ``act`` (:101-124), ``learn`` (:126-168),
``update_target_network`` (:170-172), ``save``/``load`` (:174-191) with the same
checkpoint dict and state_dict key names (conv1.weight ... fc3.bias), so
checkpoints move both ways. The network runs on evx_gemm in exact-f32 MFMA mode;
dropout stays active in ``act`` and in the target forward because the reference
never switches its networks to eval mode.

Host-side bookkeeping (the replay deque, ``random.sample``, ``np.random.random`` /
``random.randrange`` in act) consumes the global Python / numpy streams exactly
as the reference does.
"""
from __future__ import annotations

import random
from collections import OrderedDict, deque

import numpy as np
import torch

from evacx.qnet import Learner, param_shapes, layer_specs


class DQNNetwork:
    """Parameter container + forward of the reference DQNNetwork (agents/dqn_agent.py:15-61)."""

    def __init__(self, state_size=(11, 11, 6), action_size=5, hidden_size=512, _learner=None, _target=False):
        if _learner is None:
            _learner = Learner(kind="conv", device=_device(), hidden=hidden_size, actions=action_size)
        self._lr, self._target = _learner, _target
        self.training = True

    @property
    def _params(self):
        return self._lr.target if self._target else self._lr.online

    def parameters(self):
        return list(self._params.views.values())

    def named_parameters(self):
        return list(self._params.views.items())

    def state_dict(self):
        return self._params.state_dict()

    def load_state_dict(self, sd, strict=True):
        missing = [k for k in self._params.views if k not in sd]
        if strict and missing:
            raise KeyError(f"missing keys {missing}")
        self._params.load_state_dict(sd)
        self._lr.weights_written(target=self._target)  # operand copies / act table follow the weights

    def to(self, device):
        return self

    def train(self, mode=True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    def __call__(self, x):
        return self.forward(x)

    def forward(self, x):
        x = torch.as_tensor(x, dtype=torch.float32).to(self._lr.device)
        if x.dim() == 3:
            x = x.unsqueeze(0)
        return self._lr.q_values(x.contiguous(), train=self.training, target=self._target).clone()


_AGENTS = 0  # agents built in this process (distinct dropout streams)


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("evacx DQNAgent needs an MI355X (HIP) device; no CPU fallback exists")
    return torch.device("cuda", torch.cuda.current_device())


class _AdamView:
    """torch.optim.Adam-compatible state_dict() / load_state_dict() over the flat moments."""

    def __init__(self, learner: Learner):
        self._lr = learner

    @property
    def param_groups(self):
        lr = self._lr
        return [{"lr": lr.lr, "betas": lr.betas, "eps": lr.eps, "weight_decay": 0, "amsgrad": False,
                 "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                 "params": list(range(len(lr.shapes)))}]

    def state_dict(self):
        lr = self._lr
        state = {}
        if lr.adam_step > 0:
            o = 0
            for i, (k, s) in enumerate(lr.shapes.items()):
                n = int(torch.Size(s).numel())
                state[i] = {"step": torch.tensor(float(lr.adam_step)),
                            "exp_avg": lr.m[o:o + n].view(s).detach().cpu().clone(),
                            "exp_avg_sq": lr.v[o:o + n].view(s).detach().cpu().clone()}
                o += n
        return {"state": state, "param_groups": self.param_groups}

    def load_state_dict(self, sd):
        lr = self._lr
        g = sd["param_groups"][0]
        lr.lr, lr.betas, lr.eps = float(g["lr"]), tuple(g["betas"]), float(g["eps"])
        st = sd.get("state", {})
        if not st:
            lr.m.zero_()
            lr.v.zero_()
            lr.adam_step = 0
            return
        o = 0
        for i, (k, s) in enumerate(lr.shapes.items()):
            n = int(torch.Size(s).numel())
            lr.m[o:o + n].copy_(st[i]["exp_avg"].reshape(-1).to(lr.m.device))
            lr.v[o:o + n].copy_(st[i]["exp_avg_sq"].reshape(-1).to(lr.v.device))
            lr.adam_step = int(float(st[i]["step"]))
            o += n

    def zero_grad(self, set_to_none=True):
        self._lr.grads.flat.zero_()


class DQNAgent:
    """DQN agent (agents/dqn_agent.py:64-191) on the device learner."""

    def __init__(self, state_size, action_size, device, config):
        self.state_size = state_size
        self.action_size = action_size
        self.device = _device() if (device is None or torch.device(device).type != "cuda") else torch.device(device)
        self.gamma = config.get("gamma", 0.99)
        self.epsilon = config.get("epsilon", 1.0)
        self.epsilon_min = config.get("epsilon_min", 0.02)
        self.epsilon_decay = config.get("epsilon_decay", 0.9995)
        self.learning_rate = config.get("learning_rate", 0.0001)
        self.batch_size = config.get("batch_size", 32)
        self.target_update_freq = config.get("target_update_freq", 200)
        self.warmup_steps = config.get("warmup_steps", 1000)
        hidden = config.get("hidden_size", 512)
        global _AGENTS
        _AGENTS += 1
        # dropout seed: derived without drawing from any global stream (the reference's dropout
        # draws torch's generator, which a counter-based Philox cannot follow draw for draw)
        seed = (int(torch.initial_seed()) * 1000003 + _AGENTS) & 0x7FFFFFFF if config.get("seed") is None \
            else int(config["seed"])
        self._learner = Learner(kind="conv", device=self.device, lr=self.learning_rate, gamma=self.gamma,
                                max_norm=1.0, precision="f32", hidden=hidden, actions=action_size, seed=seed)
        # initial weights as the reference draws them: q_network then target_network
        # (agents/dqn_agent.py:83-84), each from torch's global generator in module order; the
        # target's draw is consumed and then overwritten by update_target_network (:95)
        if config.get("seed") is None:
            self._learner.online.init_from_global_torch()
            self._learner.target.init_from_global_torch()
        self.q_network = DQNNetwork(state_size, action_size, hidden, _learner=self._learner)
        self.target_network = DQNNetwork(state_size, action_size, hidden, _learner=self._learner, _target=True)
        self.optimizer = _AdamView(self._learner)
        self.memory = deque(maxlen=config.get("memory_size", 50000))
        self.steps = 0
        self.update_target_network()

    def remember(self, state, action, reward, next_state, done):
        self.memory.append((state, action, reward, next_state, done))

    def act(self, state, training=False):
        if training and np.random.random() <= self.epsilon:
            return random.randrange(self.action_size)
        if isinstance(state, np.ndarray):
            st = torch.from_numpy(state.astype(np.float32))
        else:
            st = torch.as_tensor(state, dtype=torch.float32)
        st = st.to(self.device)
        if st.dim() == 3:
            st = st.unsqueeze(0)
        q = self._learner.q_values(st.contiguous(), train=True)
        return np.argmax(q.cpu().numpy())

    def learn(self):
        if len(self.memory) < self.batch_size or self.steps < self.warmup_steps:
            return
        batch = random.sample(self.memory, self.batch_size)
        states, actions, rewards, next_states, dones = zip(*batch)
        dev = self.device
        s = torch.from_numpy(np.array(states, dtype=np.float32)).to(dev)
        s2 = torch.from_numpy(np.array(next_states, dtype=np.float32)).to(dev)
        a = torch.tensor([int(x) for x in actions], dtype=torch.int32, device=dev)
        r = torch.tensor(np.array(rewards, dtype=np.float64), dtype=torch.float32, device=dev)
        d = torch.tensor([bool(x) for x in dones], dtype=torch.uint8, device=dev)
        loss = self._learner.learn(s.contiguous(), a, r, d, s2.contiguous())
        if self.epsilon > self.epsilon_min:
            self.epsilon *= self.epsilon_decay
        self.steps += 1
        return loss.item()

    def update_target_network(self):
        self._learner.sync_target()

    def save(self, filepath):
        torch.save({
            "q_network": OrderedDict((k, v.cpu()) for k, v in self.q_network.state_dict().items()),
            "target_network": OrderedDict((k, v.cpu()) for k, v in self.target_network.state_dict().items()),
            "optimizer": self.optimizer.state_dict(),
            "epsilon": self.epsilon,
            "steps": self.steps,
        }, filepath)

    def load(self, filepath):
        checkpoint = torch.load(filepath, map_location="cpu", weights_only=True)
        self.q_network.load_state_dict(checkpoint["q_network"])
        self.target_network.load_state_dict(checkpoint["target_network"])
        self.optimizer.load_state_dict(checkpoint["optimizer"])
        self.epsilon = checkpoint.get("epsilon", self.epsilon_min)
        self.steps = checkpoint.get("steps", 0)


__all__ = ["DQNNetwork", "DQNAgent", "param_shapes", "layer_specs"]
