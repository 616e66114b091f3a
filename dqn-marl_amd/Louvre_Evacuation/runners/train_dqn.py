"""Single-robot DQN trainer on the device env + device learner.

Same loop as the reference's runners/train_dqn.py:29-212 (episode loop, act with
exploration, env.step, remember, learn once memory > batch, target sync every
``update_target_freq`` episodes, best/final checkpoints, reward logs), reading
``configs/dqn.yaml`` next to the Louvre_Evacuation package. Unlike the reference
module it also exports ``main``, which main.py imports.

Usage: python -m Louvre_Evacuation.main --train_dqn   (from dqn-marl_amd/)
"""
import os
import sys

project_root = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
if project_root not in sys.path:
    sys.path.insert(0, project_root)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402

from Louvre_Evacuation.agents.dqn_agent import DQNAgent  # noqa: E402
from Louvre_Evacuation.envs.evacuation_env import EvacuationEnv  # noqa: E402
from Louvre_Evacuation.utils.reward_visualizer import RewardTracker  # noqa: E402
from Louvre_Evacuation.utils.visualization import PerformanceRecorder  # noqa: E402


def load_config(config_path):
    with open(config_path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f)


def train_dqn(config_path=None, episodes=None):
    config_path = os.path.normpath(config_path or os.path.join(project_root, "configs", "dqn.yaml"))
    config = load_config(config_path)
    save_dir = os.path.join(project_root, config.get("save_path", "dqn_results"))
    os.makedirs(save_dir, exist_ok=True)
    reward_tracker = RewardTracker(save_dir=os.path.join(save_dir, "reward_logs"))
    ec = config["env"]
    env = EvacuationEnv(width=ec["width"], height=ec["height"], fire_zones=ec["fire_zones"],
                        exit_location=ec["exit_location"], num_people=ec["num_people"])
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    ac = config["agent"]
    agent = DQNAgent(env.state_size, env.action_size, device, ac)
    print(f"env {env.width}x{env.height}, {env.num_people} people, exit {env.exit_location}; "
          f"agent params {sum(p.numel() for p in agent.q_network.parameters()):,} on {agent.device}")
    episodes = config["episodes"] if episodes is None else episodes
    update_target_freq = config.get("update_target_freq", 50)
    recorder = PerformanceRecorder()
    best_reward = float("-inf")
    recent = []
    for episode in range(episodes):
        state = env.reset()
        total_reward, steps = 0, 0
        while steps < env.max_steps:
            action = agent.act(state, training=True)
            next_state, reward, done, info = env.step(action)
            agent.remember(state, action, reward, next_state, done)
            total_reward += reward
            reward_tracker.record_step(reward)
            state = next_state
            steps += 1
            if len(agent.memory) > agent.batch_size:
                agent.learn()
            if done:
                break
        if episode % update_target_freq == 0:
            agent.update_target_network()
        m = env.get_performance_metrics()
        reward_tracker.record_episode(episode=episode, total_reward=total_reward, steps=steps,
                                      evacuation_rate=m["evacuation_rate"], death_rate=m["death_rate"])
        recorder.record_episode(env, episode, total_reward)
        if total_reward > best_reward:
            best_reward = total_reward
            agent.save(os.path.join(save_dir, "best_model.pth"))
        recent = (recent + [total_reward])[-100:]
        if episode % 50 == 0 or episode == episodes - 1:
            print(f"Episode {episode:4d}: Reward={total_reward:7.2f}, Avg100={np.mean(recent):7.2f}, "
                  f"Steps={steps:3d}, Evac={m['evacuation_rate']:.2%}, Death={m['death_rate']:.2%}, "
                  f"eps={agent.epsilon:.4f}")
    agent.save(os.path.join(save_dir, "dqn_model.pth"))
    reward_tracker.save_data()
    try:
        reward_tracker.plot_reward_curves(save_path=os.path.join(save_dir, "final_reward_curves.png"), show=False)
        reward_tracker.plot_detailed_analysis(save_path=os.path.join(save_dir, "detailed_analysis.png"), show=False)
    except Exception as e:  # plotting is best-effort, as in the reference
        print(f"plotting failed: {e}")
    reward_tracker.print_statistics()
    recorder.get_dataframe().to_csv(os.path.join(save_dir, "training_performance.csv"), index=False)
    print(f"best reward {best_reward:.2f}; results in {save_dir}")
    return agent, reward_tracker


def main():
    try:
        return train_dqn()
    except KeyboardInterrupt:
        print("training interrupted")


if __name__ == "__main__":
    main()
