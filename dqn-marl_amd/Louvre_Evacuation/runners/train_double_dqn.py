"""Two independent DQN agents on EvacuationEnvMulti (reference runners/train_double_dqn.py:21-83),
on the device env and device learners."""
import csv
import os
import sys

project_root = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
if project_root not in sys.path:
    sys.path.insert(0, project_root)

import torch  # noqa: E402
import yaml  # noqa: E402

from Louvre_Evacuation.agents.dqn_agent import DQNAgent  # noqa: E402
from Louvre_Evacuation.envs.evacuation_env_multi import EvacuationEnvMulti  # noqa: E402


def train_double_dqn(episodes=200):
    with open(os.path.join(project_root, "configs", "dqn.yaml"), "r", encoding="utf-8") as f:
        cfg = yaml.safe_load(f)
    ec = cfg["env"]
    env = EvacuationEnvMulti(width=ec["width"], height=ec["height"], fire_zones=ec["fire_zones"],
                             exit_location=ec["exit_location"], num_people=ec["num_people"])
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    agents = [DQNAgent(env.state_size, env.action_size, device, cfg["agent"]) for _ in range(2)]
    logs = []
    for ep in range(episodes):
        states = env.reset()
        done, total = False, 0
        while not done:
            acts = [int(ag.act(s, training=True)) for ag, s in zip(agents, states)]
            nxt, reward, done, info = env.step(acts)
            for i, ag in enumerate(agents):
                ag.remember(states[i], acts[i], reward, nxt[i], done)
            if len(agents[0].memory) > agents[0].batch_size:
                for ag in agents:
                    ag.learn()
            states = nxt
            total += reward
        logs.append({"episode": ep, "reward": total, "evac_rate": info["evacuation_rate"],
                     "death_rate": info["death_rate"]})
        if ep % 10 == 0:
            print(f"Episode {ep}: reward={total:.2f} evac={info['evacuation_rate']:.1%} "
                  f"death={info['death_rate']:.1%}")
    save_dir = os.path.join(project_root, "dqn_results")
    os.makedirs(save_dir, exist_ok=True)
    for i, ag in enumerate(agents):
        ag.save(os.path.join(save_dir, f"double_dqn_agent{i + 1}.pth"))
    with open(os.path.join(save_dir, "double_dqn_training_log.csv"), "w", newline="", encoding="utf-8") as f:
        w = csv.DictWriter(f, fieldnames=["episode", "reward", "evac_rate", "death_rate"])
        w.writeheader()
        w.writerows(logs)
    return agents


if __name__ == "__main__":
    train_double_dqn()
