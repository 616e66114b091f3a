"""Drop-in ``EvacuationEnvMulti`` (reference envs/evacuation_env_multi.py:16-89).

Two robots starting at (10,15) and (20,15), re-placed on every reset; ``reset``
returns one observation per robot and ``step`` takes one action per robot. The
team reward is computed from robot 0, as in the reference.
"""
from __future__ import annotations

from typing import List

from .evacuation_env import EvacuationEnv


class EvacuationEnvMulti(EvacuationEnv):
    _robot_init = ((10, 15), (20, 15))
    _reset_robots = True
    _step_traj_entries = False  # the multi-robot step records only execute_move entries (:59-66)

    def __init__(self, width=36, height=30, fire_zones=None, exit_location=None, num_people=150):
        self.num_robots = len(self._robot_init)
        super().__init__(width, height, fire_zones, exit_location, num_people)

    def reset(self):
        out = super().reset()
        self.robot_trajectory = [(tuple(p), 0) for p in self.map.robot_positions]
        return out

    def _state_out(self, obs):
        return [obs[r] for r in range(obs.shape[0])]

    def _actions(self, actions: List[int]):
        assert len(actions) == self.num_robots, "one action per robot is required"
        return list(actions)

    def _record_robots(self, step0):
        for p in self.map.robot_positions:
            self.robot_trajectory.append((tuple(p), step0))

    def _info(self):
        base = super()._info()
        return {
            "robot_positions": [tuple(p) for p in self.map.robot_positions],
            "evacuation_rate": base["evacuation_rate"],
            "death_rate": base["death_rate"],
            "current_step": self.current_step,
            "simulation_time": self.time,
        }
