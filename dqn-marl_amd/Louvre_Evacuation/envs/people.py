"""Host-side view of the reference ``People`` (envs/people.py:91-314) for a device env.

``People.ROBOT_REPEL_K`` / ``ROBOT_REPEL_RANGE`` stay runtime-mutable class
attributes (envs/people.py:94-95); the device env reads them before every step.
``list`` materialises Person-like records from the device state on demand.
"""
from __future__ import annotations

import numpy as np


class People:
    ROBOT_REPEL_K: float = -20.0
    ROBOT_REPEL_RANGE: float = 5.0


class PersonView:
    __slots__ = ("id", "pos", "health", "savety", "dead", "_env", "_traj")

    def __init__(self, pid, x, y, health, flags, env=None):
        self.id = pid
        self.pos = (x + 0.5, y + 0.5)
        self.health = float(health) if not (flags & 2 and health == 0) else 0
        self.savety = bool(flags & 1)
        self.dead = bool(flags & 2)
        self._env = env
        self._traj = None

    @property
    def trajectory(self):
        """The reference's Person.trajectory (people.py:21, 52-59), built from the env's
        per-step log on first access."""
        if self._traj is None:
            self._traj = self._env.person_trajectory(self.id - 1) if self._env is not None else []
        return self._traj

    @trajectory.setter
    def trajectory(self, v):
        self._traj = v

    @property
    def speed(self):
        h = self.health
        return 0.4 if h < 20 else 1.0 * (0.3 + 0.7 * (h / 100.0))

    def name(self):
        return "ID_" + str(self.id)


class PeopleView:
    def __init__(self, env):
        self._env = env
        self._list = None
        self.tot = env.num_people

    def _invalidate(self):
        self._list = None

    @property
    def list(self):
        if self._list is None:
            h = self._env._host
            self._list = [PersonView(i + 1, int(p[0]), int(p[1]), hv, int(f), self._env)
                          for i, (p, hv, f) in enumerate(zip(h["pos"], h["health"], h["flags"]))]
        return self._list

    @property
    def rmap(self):
        return self._env._host["rmap"].astype(np.float64)

    @property
    def thmap(self):
        return self._env._host["thmap"].astype(np.float64)
