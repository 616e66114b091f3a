"""Host-side view of the reference ``Map`` (envs/map.py:37-204) for a device env.

The grid, floor field and fire tables live on the device; this object exposes the
attributes callers read or set (robot_position(s), Length, Width, Exit, space,
barrier_list, robot_range, Check_Valid, fire_model.get_max_danger). Setting a
robot position uploads it, as the reference's evaluation scripts expect.
"""
from __future__ import annotations

import numpy as np

from evacx.layout import MOVE_DX, MOVE_DY, FireSchedule

MoveTO = [np.array([dx, dy]) for dx, dy in zip(MOVE_DX, MOVE_DY)]  # envs/map.py:11-19


def Init_Barrier(A, B):
    """Normalise a barrier rectangle (envs/map.py:25-33)."""
    if A[0] > B[0]:
        A, B = B, A
    (x1, y1), (x2, y2) = A, B
    return ((x1, y1), (x2, y2)) if y1 < y2 else ((x1, y2), (x2, y1))


class _FireView:
    def __init__(self, env, spec):
        self._env = env
        self._sched = FireSchedule(spec.map_fire(), spec.additional_fire, spec.fire_max_steps)

    def get_max_danger(self, position):
        return self._sched.danger_scalar(self._env.fire_step, position)

    def update(self):  # the device advances the fire once per step
        pass


class MapView:
    def __init__(self, env):
        self._env = env
        spec = env._spec
        self.Length, self.Width = spec.L, spec.W
        self.Exit = [tuple(spec.exit)]
        self.Barrier = list(spec.barriers)
        self.robot_range = tuple(spec.robot_range)
        t = env._lay.tables
        self.space = t.floor
        self.barrier_list = [tuple(c) for c in np.argwhere(t.barrier)]
        self.fire_model = _FireView(env, spec)

    def Check_Valid(self, x, y):
        x, y = int(x), int(y)
        if x >= self.Length + 1 or x <= 0 or y >= self.Width + 1 or y <= 0:
            return False
        return bool(self._env._lay.tables.valid[x, y])

    def getDeltaP(self, P1, P2):
        return self.space[int(P1[0])][int(P1[1])] - self.space[int(P2[0])][int(P2[1])]

    def get_fire_danger(self, pos):
        return self.fire_model.get_max_danger(pos)

    @property
    def robot_position(self):
        return [int(v) for v in self._env._host["view"]]

    @robot_position.setter
    def robot_position(self, xy):
        self._env._set_view(xy)

    @property
    def robot_positions(self):
        return [[int(x), int(y)] for x, y in self._env._host["robots"]]

    @robot_positions.setter
    def robot_positions(self, positions):
        self._env._set_robots(positions)
