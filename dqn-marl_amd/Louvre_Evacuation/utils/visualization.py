"""Host-side performance log (counterpart of the reference utils/visualization.py:17-57)."""
from __future__ import annotations


class PerformanceRecorder:
    def __init__(self):
        self.episode_data = []
        self.step_data = []

    def record_episode(self, env, episode, total_reward):
        m = env.get_performance_metrics()
        self.episode_data.append({"episode": episode, "total_reward": total_reward, "evacuated": m["evacuated"],
                                  "dead": m["dead"], "remaining": m["remaining"],
                                  "evacuation_rate": m["evacuation_rate"], "death_rate": m["death_rate"],
                                  "avg_health": m["avg_health"], "min_health": m["min_health"],
                                  "total_steps": m["total_steps"]})

    def record_step(self, env, step, action, reward):
        m = env.get_performance_metrics()
        self.step_data.append({"step": step, "action": action, "reward": reward, "evacuated": m["evacuated"],
                               "dead": m["dead"], "remaining": m["remaining"], "avg_health": m["avg_health"]})

    def get_dataframe(self):
        import pandas as pd
        return pd.DataFrame(self.episode_data)


def visualize_trajectories(env, save_path=None):
    """Robot trajectory + final people positions (matplotlib, non-interactive)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots(figsize=(6, 5))
    rt = [p for p, _ in env.robot_trajectory]
    if rt:
        ax.plot([p[0] for p in rt], [p[1] for p in rt], "b-", lw=1)
    ppl = env.people.list
    ax.scatter([p.pos[0] for p in ppl], [p.pos[1] for p in ppl], s=4,
               c=["g" if p.savety else ("k" if p.dead else "r") for p in ppl])
    ax.set_xlim(0, env.width + 2)
    ax.set_ylim(0, env.height + 2)
    if save_path:
        fig.savefig(save_path, dpi=100)
    plt.close(fig)
