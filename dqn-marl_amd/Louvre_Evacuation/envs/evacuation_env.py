"""Drop-in ``EvacuationEnv`` backed by the HIP env kernels (libevacx.so).

Mirrors the public API of the reference's ``envs/evacuation_env.py`` (constructor
:21-59, ``reset`` :61-82, ``step`` :122-172, ``get_performance_metrics`` :290-309,
class-level reward coefficients :16-19). The step itself runs on the GPU
(evacx.env.VecEnv with E=1). The reference draws from the *global* CPython
``random`` and legacy ``numpy.random`` generators; this wrapper hands both MT19937
states to the device before every reset/step and takes them back afterwards, so a
script that mixes env steps with its own random draws consumes exactly the same
streams as it would with the reference.
"""
from __future__ import annotations

import random
from typing import Dict, Tuple

import numpy as np
import torch

from evacx.env import DeviceLayout, VecEnv, pack_xy
from evacx.layout import FireSchedule, LayoutSpec, build_tables_device

from .map import MapView
from .people import People, PeopleView

_LAYOUTS: Dict[Tuple, DeviceLayout] = {}


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("evacx EvacuationEnv needs an MI355X (HIP) device; no CPU fallback exists")
    return torch.device("cuda", torch.cuda.current_device())


def device_layout(spec: LayoutSpec, P: int) -> DeviceLayout:
    key = (spec.L, spec.W, tuple(spec.exit), tuple(map(tuple, spec.robot_init)), spec.reset_robots,
           tuple(spec.reset_view), P)
    lay = _LAYOUTS.get(key)
    if lay is None:
        dev = _device()
        lay = DeviceLayout(build_tables_device([spec], device=dev)[0], P, device=dev)
        _LAYOUTS[key] = lay
    return lay


def _get_py_state() -> np.ndarray:
    st = random.getstate()
    return np.array(st[1], dtype=np.uint64).astype(np.uint32)


def _set_py_state(words: np.ndarray, gauss_next=None):
    """Install the MT words back into the global stream. ``gauss_next`` (random.gauss's
    cached second variate) is not touched by the env, so the caller's value is kept."""
    v = [int(x) for x in words]
    random.setstate((3, tuple(v), gauss_next))


def _action_code(x) -> int:
    """Map an action to the device code as Map.move_robot tests it (envs/map.py:180-193):
    Python equality with 0..4 (so 3.0, np.float64(1), True or a 0-d array move the robot),
    anything else is ignored (-1)."""
    if x in (0, 1, 2, 3, 4):
        return next(v for v in range(5) if x == v)
    return -1


def _get_np_state():
    return np.random.get_state()


def _np_words(st) -> np.ndarray:
    return np.concatenate([np.asarray(st[1], np.uint32), np.array([st[2]], np.uint32)])


class EvacuationEnv:
    """Single-robot evacuation environment (reference envs/evacuation_env.py)."""

    EVAC_REWARD: float = 50.0
    DEATH_PENALTY: float = 200.0
    DEATH_ACC_PENALTY: float = 0.5
    ALIVE_BONUS: float = 1.0

    _robot_init = ((15, 15),)
    _reset_robots = False

    def __init__(self, width=36, height=30, fire_zones=None, exit_location=None, num_people=150):
        self.width = width
        self.height = height
        self.num_people = num_people
        self.time_per_step = 0.5
        self.max_simulation_time = 600
        self.max_steps = int(self.max_simulation_time / self.time_per_step)
        if exit_location is None:
            exit_location = [36, 15]
        if fire_zones is None:
            fire_zones = {(18, 14), (19, 14), (20, 14), (18, 15), (19, 15), (20, 15), (18, 16), (19, 16), (20, 16)}
        self.exit_location = exit_location
        self.fire_zones = fire_zones  # stored, never affects physics (as in the reference)
        self.state_size = (11, 11, 6)
        self.action_size = 5
        init = tuple(tuple(p) for p in self._robot_init)
        self._spec = LayoutSpec(L=width, W=height, exit=(int(exit_location[0]), int(exit_location[1])),
                                robot_init=init, reset_robots=self._reset_robots,
                                reset_view=(15, 15) if not self._reset_robots else init[0])
        self._lay = device_layout(self._spec, num_people)
        self._venv = VecEnv(self._lay, 1, thmap=True)
        self._fire_env = FireSchedule(self._spec.env_fire(), self._spec.additional_fire, self._spec.fire_max_steps)
        self.map = MapView(self)
        self.people = PeopleView(self)
        self.robot_direction = 1
        self._host = None
        self.reset()

    # ----------------------------------------------------------- plumbing
    def _push_rng(self):
        self._np_state = _get_np_state()
        self._gauss_next = random.getstate()[2]
        self._venv.set_rng(_get_py_state()[None], _np_words(self._np_state)[None])

    def _pull_rng(self):
        py, nps = self._venv.get_rng()
        _set_py_state(py[0], self._gauss_next)
        st = self._np_state
        np.random.set_state((st[0], nps[0][:624].copy(), int(nps[0][624]), st[3], st[4]))

    def _sync_params(self):
        cls = type(self)
        self._lay.set_params(evac_reward=cls.EVAC_REWARD, death_penalty=cls.DEATH_PENALTY,
                             death_acc_penalty=cls.DEATH_ACC_PENALTY, alive_bonus=cls.ALIVE_BONUS,
                             repel_k=People.ROBOT_REPEL_K, repel_range=People.ROBOT_REPEL_RANGE)

    def _refresh(self):
        self._host = self._venv.host_state(0)
        sc = self._host["scal"]
        self.current_step = int(sc[1])
        self.time = 0.5 * self.current_step if self.current_step else 0
        self.prev_evacuated = int(sc[2])
        self.prev_dead = int(sc[3])
        self.people._invalidate()

    @property
    def fire_step(self) -> int:
        return int(self._host["scal"][0])

    def _obs(self) -> np.ndarray:
        obs = self._venv.expand_obs(torch.float64).cpu().numpy()[0]  # [R, 11, 11, 6]
        # channel 2 outside the device danger table (only for externally moved robots)
        for r in range(obs.shape[0]):
            cx, cy = (self._host["view"] if r == 0 else self._host["robots"][r])
            if not (0 <= cx <= self.width + 1 and 0 <= cy <= self.height + 1):
                for i in range(11):
                    for j in range(11):
                        obs[r, i, j, 2] = self._fire_env.danger_scalar(self.fire_step, (cx + i - 5, cy + j - 5))
        return obs

    # --------------------------------------------------------------- API
    def reset(self):
        self._push_rng()
        self._venv.reset()
        self._pull_rng()
        self._refresh()
        # person trajectories (evacuation_env.py:79-80): one log entry per step, materialised on access
        self._traj_log = [self._host["pos"].copy()]
        self.time = 0
        self.robot_direction = 1
        self.robot_trajectory = [(tuple(self.map.robot_position), 0)]
        return self._state_out(self._obs())

    def _state_out(self, obs):
        return obs[0]

    def _actions(self, action):
        return [action]

    def _patrol(self, rid: int):
        """Map.move_robot(None) (envs/map.py:172-178): robot rid steps one cell along x,
        turning at the ends of map.robot_range; no validity check. The direction lives on the
        map (unset until a robot first reaches an end, as in the reference). The move is made
        here and the device step sees action -1 for this robot (no move)."""
        pos = self.map.robot_positions
        x = pos[rid][0]
        if x >= self.map.robot_range[1]:
            self.map.robot_direction = -1
        elif x <= self.map.robot_range[0]:
            self.map.robot_direction = 1
        pos[rid][0] = x + self.map.robot_direction
        self._set_robots(pos)
        if rid == 0:  # map.robot_position = robot_positions[0]
            self._set_view(pos[0])

    def step(self, action):
        acts = self._actions(action)
        codes = []
        for rid, x in enumerate(acts):  # robots move in id order (evacuation_env_multi.py:60-61)
            if x is None:
                self._patrol(rid)
                codes.append(-1)
            else:
                codes.append(_action_code(x))
        a = np.array(codes, dtype=np.int32)
        self._sync_params()
        step0 = self.current_step
        self._push_rng()
        self._venv.step(torch.from_numpy(a).to(self._venv.pk.device))
        self._pull_rng()
        prev = self._host["pos"]
        self._refresh()
        cur = self._host["pos"].copy()
        # execute_move records every mover (people.py:303-306); a person moves to a neighbour
        self._traj_log.append((step0, cur, (cur != prev).any(axis=1), self._host["health"].copy()))
        self.time = 0.5 * self.current_step
        reward = float(self._venv.reward[0].item())
        done = bool(self._venv.done[0].item())
        self._record_robots(step0)
        return self._state_out(self._obs()), reward, done, self._info()

    _step_traj_entries = True  # EvacuationEnv.step appends {'pos', 'step'} per person (:134-135)

    def person_trajectory(self, i: int) -> list:
        """Person i's ``trajectory`` list as the reference builds it: the reset entry
        (evacuation_env.py:79-80), then per step the execute_move record of a mover
        (people.py:52-59, 306: savety/dead still False when recorded) and, in the single-robot
        env, the per-step entry (evacuation_env.py:134-135)."""
        log = self._traj_log
        p0 = log[0][i]
        out = [{"pos": (int(p0[0]) + 0.5, int(p0[1]) + 0.5), "step": 0}]
        for step0, cur, moved, health in log[1:]:
            pos = (int(cur[i][0]) + 0.5, int(cur[i][1]) + 0.5)
            if moved[i]:
                out.append({"pos": pos, "health": float(health[i]), "savety": False, "dead": False})
            if self._step_traj_entries:
                out.append({"pos": pos, "step": step0})
        return out

    def _record_robots(self, step0):
        self.robot_trajectory.append((tuple(self.map.robot_position), step0))

    def _info(self):
        ppl = self.people.list
        ev = int((self._host["flags"] & 1).sum())
        de = int(((self._host["flags"] >> 1) & 1).sum())
        return {
            "robot_position": tuple(self.map.robot_position),
            "people_positions": [p.pos for p in ppl],
            "health_values": [p.health for p in ppl],
            "evacuation_status": [p.savety for p in ppl],
            "fire_spread": [],
            "evacuation_rate": ev / self.num_people,
            "death_rate": de / self.num_people,
            "current_step": self.current_step,
            "simulation_time": self.time,
        }

    def get_performance_metrics(self):
        fl = self._host["flags"]
        h = self._host["health"]
        evacuated = int((fl & 1).sum())
        dead = int(((fl >> 1) & 1).sum())
        alive_h = [float(x) for x, f in zip(h, fl) if not (f & 2)]
        return {
            "evacuated": evacuated,
            "dead": dead,
            "remaining": self.num_people - evacuated - dead,
            "evacuation_rate": evacuated / self.num_people,
            "death_rate": dead / self.num_people,
            "avg_health": np.mean(alive_h),
            "min_health": min(alive_h, default=100),
            "total_steps": self.current_step,
            "total_time": self.time,
        }

    def _set_view(self, xy):
        self._venv.view[0] = int(pack_xy(int(xy[0]), int(xy[1])))
        self._host["view"] = np.array([int(xy[0]), int(xy[1])], np.int32)

    def _set_robots(self, positions):
        pos = [list(p) for p in positions]
        R = self._lay.R
        if len(pos) < R:
            pos = pos + [[15, 15]] * (R - len(pos))
        v = pack_xy([p[0] for p in pos[:R]], [p[1] for p in pos[:R]])
        self._venv.robots.copy_(torch.from_numpy(v).to(self._venv.robots.device))
        self._host["robots"] = np.array(pos[:R], np.int32)
