"""Value-mixing learn step of the reference's two-robot trainer on the device learners.

Reference: Louvre_Evacuation/runners/train_qmix.py. Its
``MixingNetwork`` (:39-54) mixes the chosen-action Q values of n agents with
absolute-valued weights (n -> embed -> 1, ReLU between), and each learn step (:78-118)
is: per-agent online Q gathered at the taken actions, target Q_tot from the target
agents' max Q through the target mixer, MSE, one backward through mixer and agents,
``clip_grad_norm_(1.0)`` per parameter set, one Adam step each.

Here every agent's network runs on its ``evacx.qnet.Learner`` (forward, backward,
fused clip + Adam on the device); only the mixer -- 2 x 32 + 32 + 32 + 1 parameters --
stays a torch module on the same device, as in the reference. d loss / d q_i from the
mixer's autograd is scattered into each agent's dQ at its taken action and handed to
the agent's own backward.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .qnet import Learner


class MixingNetwork(torch.nn.Module):
    """runners/train_qmix.py:39-54: q_tot = relu(q @ |W1| + b1) @ |W2| + b2."""

    def __init__(self, n_agents: int, embed_dim: int = 32):
        super().__init__()
        self.n_agents = n_agents
        self.embed_dim = embed_dim
        self.fc1_weight = torch.nn.Parameter(torch.randn(n_agents, embed_dim))
        self.fc1_bias = torch.nn.Parameter(torch.zeros(embed_dim))
        self.fc2_weight = torch.nn.Parameter(torch.randn(embed_dim, 1))
        self.fc2_bias = torch.nn.Parameter(torch.zeros(1))

    def forward(self, q_vals: torch.Tensor) -> torch.Tensor:  # (batch, n_agents) -> (batch,)
        w1 = torch.abs(self.fc1_weight)
        w2 = torch.abs(self.fc2_weight)
        hidden = torch.relu(torch.matmul(q_vals, w1) + self.fc1_bias)
        return (torch.matmul(hidden, w2) + self.fc2_bias).squeeze(-1)


class QMixLearnStep:
    """One learn step over n agents' device learners + a torch mixer (see module doc)."""

    def __init__(self, learners: Sequence[Learner], mixing: MixingNetwork, target_mixing: MixingNetwork,
                 mix_optimizer: torch.optim.Optimizer, gamma: float = 0.99, max_norm: float = 1.0):
        self.learners: List[Learner] = list(learners)
        self.mixing, self.target_mixing, self.mix_opt = mixing, target_mixing, mix_optimizer
        self.gamma, self.max_norm = gamma, max_norm

    def __call__(self, states: Sequence[torch.Tensor], actions: Sequence[torch.Tensor], reward: torch.Tensor,
                 done: torch.Tensor, next_states: Sequence[torch.Tensor],
                 masks: Optional[Sequence[torch.Tensor]] = None,
                 target_masks: Optional[Sequence[torch.Tensor]] = None) -> torch.Tensor:
        """states[i]: [B, 11, 11, 6] f32 of agent i; actions[i]: [B] int; reward [B] f32;
        done [B] bool/uint8; masks / target_masks: optional dropout keep-masks [B, hidden]
        (default: drawn by each learner, dropout active as in the reference)."""
        B = reward.shape[0]
        qs, qts = [], []
        for i, lr in enumerate(self.learners):
            m = masks[i] if masks is not None else lr.dropout_mask(B, "on")
            mt = target_masks[i] if target_masks is not None else lr.dropout_mask(B, "tg")
            Q = lr.net.forward(states[i].contiguous(), m, save=True)
            qs.append(Q.gather(1, actions[i].long().view(B, 1)).view(B).clone())
            qts.append(lr.tnet.forward(next_states[i].contiguous(), mt, save=False, tag="t_").max(1)[0].clone())
        with torch.no_grad():  # y_tot = r + gamma * Q_tot'(s') * ~done (:98-103)
            y = reward.float() + self.gamma * self.target_mixing(torch.stack(qts, 1)) * (~done.bool()).float()
        q_cat = torch.stack(qs, 1).detach().requires_grad_(True)
        loss = torch.nn.functional.mse_loss(self.mixing(q_cat), y)
        self.mix_opt.zero_grad()
        loss.backward()
        for i, lr in enumerate(self.learners):  # d loss / d Q_i at the taken action only
            dQ = torch.zeros(B, lr.actions, dtype=torch.float32, device=q_cat.device)
            dQ.scatter_(1, actions[i].long().view(B, 1), q_cat.grad[:, i:i + 1].float())
            lr.net.backward(dQ, lr.grads)
            lr.step_optimizer()  # clip_grad_norm_(agent, 1.0) + Adam (:110-113)
        torch.nn.utils.clip_grad_norm_(self.mixing.parameters(), self.max_norm)
        self.mix_opt.step()
        return loss.detach()

    def sync_targets(self):
        """agent.update_target_network() for every agent + target_mixing <- mixing (:116-118)."""
        for lr in self.learners:
            lr.sync_target()
        self.target_mixing.load_state_dict(self.mixing.state_dict())
