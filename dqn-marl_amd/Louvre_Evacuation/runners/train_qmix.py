"""Two-robot value-mixing trainer (reference runners/train_qmix.py:25-134) on the device
env and the device learners: the same episode loop, replay deque of joint transitions,
random.sample batches, mixing network with absolute-valued weights, per-parameter-set
clip_grad_norm_(1.0) + Adam, stochastic target sync, CSV log and saved agents. The
learn step itself is evacx.qmix.QMixLearnStep: the agents' networks forward and
backward on the GPU kernels (the reference calls q_network under torch autograd), the
2 -> 32 -> 1 mixer stays a torch module.
"""
import csv
import os
import random
import sys
from collections import deque

project_root = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
if project_root not in sys.path:
    sys.path.insert(0, project_root)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402
from torch.optim.adam import Adam  # noqa: E402

from evacx.qmix import MixingNetwork, QMixLearnStep  # noqa: E402
from Louvre_Evacuation.agents.dqn_agent import DQNAgent  # noqa: E402
from Louvre_Evacuation.envs.evacuation_env_multi import EvacuationEnvMulti  # noqa: E402


def load_cfg():
    with open(os.path.join(project_root, "configs", "dqn.yaml"), "r", encoding="utf-8") as f:
        return yaml.safe_load(f)


def train_qmix(episodes=200):
    cfg = load_cfg()
    ec = cfg["env"]
    env = EvacuationEnvMulti(width=ec["width"], height=ec["height"], fire_zones=ec["fire_zones"],
                             exit_location=ec["exit_location"], num_people=ec["num_people"])
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    agent_cfg = cfg["agent"]
    agent1 = DQNAgent(env.state_size, env.action_size, device, agent_cfg)
    agent2 = DQNAgent(env.state_size, env.action_size, device, agent_cfg)
    gamma = agent_cfg.get("gamma", 0.99)
    replay = deque(maxlen=5000)
    dev = agent1.device
    mixing = MixingNetwork(n_agents=2).to(dev)
    target_mixing = MixingNetwork(n_agents=2).to(dev)
    target_mixing.load_state_dict(mixing.state_dict())
    mix_optimizer = Adam(mixing.parameters(), lr=1e-3)
    step = QMixLearnStep([agent1._learner, agent2._learner], mixing, target_mixing, mix_optimizer, gamma=gamma)
    logs = []
    info = {"evacuation_rate": 0.0, "death_rate": 0.0}
    for ep in range(episodes):
        states = env.reset()
        done = False
        total_reward = 0
        while not done:
            a1 = int(agent1.act(states[0], training=True))
            a2 = int(agent2.act(states[1], training=True))
            next_states, reward, done, info = env.step([a1, a2])
            replay.append((states, [a1, a2], reward, next_states, done))
            states = next_states
            total_reward += reward
            if len(replay) >= agent1.batch_size:
                batch = random.sample(replay, agent1.batch_size)
                s = [torch.from_numpy(np.array([b[0][i] for b in batch], dtype=np.float32)).to(dev) for i in range(2)]
                a = [torch.tensor([b[1][i] for b in batch], dtype=torch.int64, device=dev) for i in range(2)]
                r = torch.tensor(np.array([b[2] for b in batch], dtype=np.float32), device=dev)
                ns = [torch.from_numpy(np.array([b[3][i] for b in batch], dtype=np.float32)).to(dev)
                      for i in range(2)]
                d = torch.tensor([bool(b[4]) for b in batch], dtype=torch.bool, device=dev)
                step(s, a, r, d, ns)
                if random.random() < 0.01:
                    step.sync_targets()
        logs.append({"episode": ep, "reward": total_reward, "evac_rate": info["evacuation_rate"],
                     "death_rate": info["death_rate"]})
        if ep % 10 == 0:
            print(f"QMIX Episode {ep}: reward={total_reward:.1f} evac={info['evacuation_rate']:.1%} "
                  f"death={info['death_rate']:.1%}")
    save_dir = os.path.join(project_root, "dqn_results")
    os.makedirs(save_dir, exist_ok=True)
    agent1.save(os.path.join(save_dir, "qmix_agent1.pth"))
    agent2.save(os.path.join(save_dir, "qmix_agent2.pth"))
    with open(os.path.join(save_dir, "qmix_training_log.csv"), "w", newline="", encoding="utf-8") as f:
        w = csv.DictWriter(f, fieldnames=["episode", "reward", "evac_rate", "death_rate"])
        w.writeheader()
        w.writerows(logs)
    print("QMIX training done: models and log saved")
    return agent1, agent2, mixing


if __name__ == "__main__":
    train_qmix()
