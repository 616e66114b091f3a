"""Host-side reward log (counterpart of the reference utils/reward_visualizer.py:18-310).

Same methods and output files (reward_data.json, episode_data.csv, two PNG
plots); plotting uses a non-interactive matplotlib backend and is optional.
"""
from __future__ import annotations

import json
import os
from collections import deque

import numpy as np


class RewardTracker:
    def __init__(self, save_dir="reward_logs"):
        self.save_dir = save_dir
        os.makedirs(save_dir, exist_ok=True)
        self.episode_rewards, self.episode_steps = [], []
        self.episode_evacuation_rates, self.episode_death_rates = [], []
        self.step_rewards = []
        self.window_size = 100
        self.recent_rewards = deque(maxlen=self.window_size)
        self.total_episodes = 0
        self.total_steps = 0

    def record_episode(self, episode, total_reward, steps, evacuation_rate, death_rate):
        self.episode_rewards.append(float(total_reward))
        self.episode_steps.append(int(steps))
        self.episode_evacuation_rates.append(float(evacuation_rate))
        self.episode_death_rates.append(float(death_rate))
        self.recent_rewards.append(float(total_reward))
        self.total_episodes = episode + 1
        self.total_steps += steps

    def record_step(self, reward):
        self.step_rewards.append(float(reward))

    def get_recent_average(self):
        return float(np.mean(self.recent_rewards)) if self.recent_rewards else 0

    def get_statistics(self):
        if not self.episode_rewards:
            return {}
        r = np.asarray(self.episode_rewards)
        return {"total_episodes": self.total_episodes, "total_steps": self.total_steps,
                "avg_reward": float(r.mean()), "max_reward": float(r.max()), "min_reward": float(r.min()),
                "std_reward": float(r.std()), "recent_avg_reward": self.get_recent_average(),
                "avg_evacuation_rate": float(np.mean(self.episode_evacuation_rates)),
                "avg_death_rate": float(np.mean(self.episode_death_rates)),
                "avg_steps_per_episode": float(np.mean(self.episode_steps))}

    def print_statistics(self):
        s = self.get_statistics()
        if not s:
            print("no statistics yet")
            return
        print(f"episodes: {s['total_episodes']}  steps: {s['total_steps']}")
        print(f"reward avg {s['avg_reward']:.2f} max {s['max_reward']:.2f} min {s['min_reward']:.2f} "
              f"std {s['std_reward']:.2f} recent{self.window_size} {s['recent_avg_reward']:.2f}")
        print(f"evacuation {s['avg_evacuation_rate']:.2%}  death {s['avg_death_rate']:.2%}  "
              f"steps/episode {s['avg_steps_per_episode']:.1f}")

    def save_data(self):
        data = {"episode_rewards": self.episode_rewards, "episode_steps": self.episode_steps,
                "episode_evacuation_rates": self.episode_evacuation_rates,
                "episode_death_rates": self.episode_death_rates, "step_rewards": self.step_rewards,
                "statistics": self.get_statistics()}
        with open(os.path.join(self.save_dir, "reward_data.json"), "w", encoding="utf-8") as f:
            json.dump(data, f, ensure_ascii=False, indent=2)
        with open(os.path.join(self.save_dir, "episode_data.csv"), "w", encoding="utf-8") as f:
            f.write("episode,reward,steps,evacuation_rate,death_rate\n")
            for i, row in enumerate(zip(self.episode_rewards, self.episode_steps, self.episode_evacuation_rates,
                                        self.episode_death_rates)):
                f.write(",".join(str(v) for v in (i,) + row) + "\n")

    def load_data(self, filepath):
        with open(filepath, "r", encoding="utf-8") as f:
            d = json.load(f)
        self.episode_rewards = d["episode_rewards"]
        self.episode_steps = d["episode_steps"]
        self.episode_evacuation_rates = d["episode_evacuation_rates"]
        self.episode_death_rates = d["episode_death_rates"]
        self.step_rewards = d["step_rewards"]
        self.recent_rewards = deque(self.episode_rewards[-self.window_size:], maxlen=self.window_size)
        self.total_episodes = len(self.episode_rewards)
        self.total_steps = int(sum(self.episode_steps))

    def _plot(self, save_path, show, panels):
        import matplotlib
        if not show:
            matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig, axes = plt.subplots(1, len(panels), figsize=(6 * len(panels), 4))
        for ax, (title, ys) in zip(np.atleast_1d(axes), panels):
            ax.plot(ys)
            ax.set_title(title)
        fig.tight_layout()
        if save_path:
            fig.savefig(save_path, dpi=100)
        if show:
            plt.show()
        plt.close(fig)

    def plot_reward_curves(self, save_path=None, show=True):
        self._plot(save_path, show, [("episode reward", self.episode_rewards), ("step reward", self.step_rewards)])

    def plot_detailed_analysis(self, save_path=None, show=True):
        self._plot(save_path, show, [("evacuation rate", self.episode_evacuation_rates),
                                     ("death rate", self.episode_death_rates), ("steps", self.episode_steps)])
