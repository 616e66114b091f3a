#!/usr/bin/env python3
"""Drop-in ``runners/evaluate_strategies.py``: no robot vs a static robot vs a trained DQN
robot on the device env (reference runners/evaluate_strategies.py:34-165).

Same functions and command line as the reference -- ``build_env_from_config`` (:34-44),
``evaluate`` (:47-75), ``no_robot_policy`` (:79-85), ``static_robot_policy`` (:88-90),
``build_dqn_policy`` (:93-110), ``main`` (:115-161) -- so a checkpoint written by either
framework's ``DQNAgent.save`` is evaluated the same way.
"""
import argparse
import os
import sys

import numpy as np
import torch
import yaml

project_root = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
if project_root not in sys.path:
    sys.path.insert(0, project_root)

from Louvre_Evacuation.agents.dqn_agent import DQNAgent  # noqa: E402
from Louvre_Evacuation.envs.evacuation_env import EvacuationEnv  # noqa: E402


def build_env_from_config(cfg):
    """EvacuationEnv from a config dict's ``env`` (or ``environment``) section."""
    e = cfg["env"] if "env" in cfg else cfg.get("environment", {})
    return EvacuationEnv(width=e.get("width", 36), height=e.get("height", 30), fire_zones=e.get("fire_zones"),
                         exit_location=e.get("exit_location"), num_people=e.get("num_people", 150))


def evaluate(env_builder, policy_fn, episodes):
    """Run ``episodes`` fresh envs to completion under ``policy_fn(state, env)``; mean of the
    final avg_health and total_time over the episodes, plus every episode's metrics."""
    records = []
    for _ in range(episodes):
        env = env_builder()
        state, done = env.reset(), False
        while not done:
            state, _, done, _ = env.step(policy_fn(state, env))
        records.append(env.get_performance_metrics())
    return {"records": records,
            "avg_health": np.mean([m["avg_health"] for m in records]),
            "avg_time": np.mean([m["total_time"] for m in records])}


def no_robot_policy(state, env):
    """No robot: the robot is moved far away once per env and then stays (action 4)."""
    if getattr(env, "_no_robot_shifted", False) is False:
        env.map.robot_position = [1000, 1000]
        env._no_robot_shifted = True
    return 4


def static_robot_policy(state, env):
    """Static robot: always stays where it is (action 4)."""
    return 4


def build_dqn_policy(model_path, device, env_sample):
    """Greedy policy of a trained DQNAgent loaded from ``model_path`` (epsilon 0; the
    network keeps the reference's train-mode dropout in act)."""
    agent = DQNAgent(env_sample.state_size, env_sample.action_size, device,
                     {"gamma": 0.99, "epsilon": 0.0, "epsilon_min": 0.0, "epsilon_decay": 1.0,
                      "learning_rate": 1e-4, "batch_size": 32, "memory_size": 10000})
    agent.load(model_path)
    agent.epsilon = 0.0

    def _policy(state, _env):
        return agent.act(state)

    return _policy


def main(argv=None):
    ap = argparse.ArgumentParser(description="no robot vs static robot vs DQN robot")
    ap.add_argument("--config", default=os.path.join(project_root, "configs", "dqn.yaml"))
    ap.add_argument("--model_path", default=os.path.join(project_root, "dqn_results", "best_model.pth"))
    ap.add_argument("--episodes", type=int, default=20)
    args = ap.parse_args(argv)
    cfg = {}
    if os.path.exists(args.config):
        with open(args.config, "r", encoding="utf-8") as f:
            cfg = yaml.safe_load(f)
    env_builder = lambda: build_env_from_config(cfg)  # noqa: E731
    env_sample = env_builder()
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    rows = []
    for name, pol in [("no robot", no_robot_policy), ("static robot (15,15)", static_robot_policy)]:
        r = evaluate(env_builder, pol, args.episodes)
        print(f"\n=== {name} ===\navg health {r['avg_health']:.2f}, avg evacuation time {r['avg_time']:.1f}s")
        rows.append((name, r))
    if not os.path.exists(args.model_path):
        print(f"DQN model not found: {args.model_path}; DQN evaluation skipped.")
        return rows
    r = evaluate(env_builder, build_dqn_policy(args.model_path, device, env_sample), args.episodes)
    print(f"\n=== DQN robot ===\navg health {r['avg_health']:.2f}, avg evacuation time {r['avg_time']:.1f}s")
    rows.append(("DQN robot", r))
    print("\n=== summary ===\npolicy\t\tavg health\tavg time (s)")
    for name, r in rows:
        print(f"{name}\t{r['avg_health']:.2f}\t\t{r['avg_time']:.1f}")
    return rows


if __name__ == "__main__":
    main()
