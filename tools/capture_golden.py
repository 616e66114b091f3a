#!/usr/bin/env python3
"""Capture golden fixtures from the reference (run ONLY in the build container).

This script imports the read-only reference (``/root/reference``) to generate
input/output vectors; the reference itself never travels to the GPU box. The
outputs are small ``.npz`` files under ``tests/golden/`` that pin

* the static layout tables the reference builds (floor field after
  ``Map.Init_Potential`` -- ``envs/map.py:127-148``; validity -- ``Map.Check_Valid``
  ``envs/map.py:85-92``; exit cells -- ``Map.checkSavefy`` ``envs/map.py:93-113``),
* the fire danger tables, i.e. ``FireSpreadModel.get_max_danger`` evaluated at
  person positions (cell centres, ``envs/people.py:205``) and at observation
  coordinates (integer cells, ``envs/evacuation_env.py:106``) for every fire step,
  because those values run through ``numpy.exp`` (``envs/fire_model.py:183``),
* whole trajectories of ``EvacuationEnv`` / ``EvacuationEnvMulti``
  (``envs/evacuation_env.py:61-172``, ``envs/evacuation_env_multi.py:38-89``)
  started from recorded MT19937 states of Python ``random`` and legacy
  ``numpy.random`` (the two streams the reference consumes),
* ``DQNNetwork`` forward outputs and ``DQNAgent.learn`` results
  (``agents/dqn_agent.py:15-168``) for deterministic, closed-form weights.

Usage:  PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tools/capture_golden.py
"""
import hashlib
import os
import random
import sys

import numpy as np

REF = os.environ.get("EVX_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

from Louvre_Evacuation.envs.evacuation_env import EvacuationEnv  # noqa: E402
from Louvre_Evacuation.envs.evacuation_env_multi import EvacuationEnvMulti  # noqa: E402
from Louvre_Evacuation.envs.fire_model import FireSpreadModel, FireSource  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
OBS_PAD = 5  # observation window half-width (envs/evacuation_env.py:92-94)


class EvacuationEnvMultiR(EvacuationEnvMulti):
    """EvacuationEnvMulti generalised from 2 hard-coded robots to R robots.

    Only the robot count and the reset positions change; every method body of
    the reference is inherited unchanged except the two places that hard-code
    ``[[10, 15], [20, 15]]`` (``envs/evacuation_env_multi.py:21,27,35``).
    """

    def __init__(self, robot_init, **kw):
        self._robot_init = [list(p) for p in robot_init]
        self.num_robots = len(robot_init)
        EvacuationEnv.__init__(self, **kw)
        self.map.robot_positions = [list(p) for p in self._robot_init]
        self.map.robot_position = self.map.robot_positions[0]

    def reset(self):
        EvacuationEnv.reset(self)
        self.map.robot_positions = [list(p) for p in self._robot_init]
        self.map.robot_position = self.map.robot_positions[0]
        self.robot_trajectory = [(tuple(p), 0) for p in self.map.robot_positions]
        return self._get_joint_state()


# ----------------------------------------------------------------------------
# state extraction
# ----------------------------------------------------------------------------

def rng_states():
    st = random.getstate()
    assert st[0] == 3
    py = np.array(st[1], dtype=np.uint64).astype(np.uint32)  # 624 words + index
    name, keys, pos, has_gauss, _ = np.random.get_state()
    assert name == "MT19937" and has_gauss == 0
    npk = np.concatenate([np.asarray(keys, dtype=np.uint32), np.array([pos], dtype=np.uint32)])
    return py, npk


def env_state(env):
    ppl = env.people.list
    pos = np.array([[int(p.pos[0]), int(p.pos[1])] for p in ppl], dtype=np.int32)
    # every recorded position must be a cell centre (x + 0.5, y + 0.5)
    for p in ppl:
        assert p.pos[0] - int(p.pos[0]) == 0.5 and p.pos[1] - int(p.pos[1]) == 0.5
    health = np.array([float(p.health) for p in ppl], dtype=np.float64)
    acc = np.array([float(p.move_accumulator) for p in ppl], dtype=np.float64)
    flags = np.array([(1 if p.savety else 0) | (2 if p.dead else 0) for p in ppl], dtype=np.uint8)
    rmap = np.asarray(env.people.rmap, dtype=np.float64)
    assert np.all((rmap == 0) | (rmap == 1))
    thmap = np.asarray(env.people.thmap, dtype=np.float64)
    assert np.all(thmap == np.round(thmap))
    robots = np.array(env.map.robot_positions, dtype=np.int32).reshape(-1, 2)
    view = np.array(env.map.robot_position, dtype=np.int32)
    fs_env = env.fire_model.progressive_model.current_step
    fs_map = env.map.fire_model.progressive_model.current_step
    assert fs_env == fs_map
    return dict(pos=pos, health=health, acc=acc, flags=flags, rmap=rmap.astype(np.uint8),
                thmap=thmap.astype(np.int32), robots=robots, view=view,
                fire_step=np.int32(fs_env), time=np.float64(env.time),
                cur_step=np.int32(env.current_step), prev_evac=np.int32(env.prev_evacuated),
                prev_dead=np.int32(env.prev_dead))


FIELDS = ["pos", "health", "acc", "flags", "rmap", "thmap", "robots", "view", "obs"]


def canon_bytes(name, a):
    """Canonical serialisation shared with tests/golden_util.py."""
    dt = {"pos": np.int32, "health": np.float64, "acc": np.float64, "flags": np.uint8,
          "rmap": np.uint8, "thmap": np.int32, "robots": np.int32, "view": np.int32,
          "obs": np.float64}[name]
    return np.ascontiguousarray(np.asarray(a, dtype=dt)).tobytes()


def digest(name, a):
    return np.frombuffer(hashlib.sha256(canon_bytes(name, a)).digest(), dtype=np.uint8)


# ----------------------------------------------------------------------------
# layout tables
# ----------------------------------------------------------------------------

def layout_tables(env_kwargs, t_max):
    """Tables of one layout, from a throw-away env (consumes RNG: call before seeding)."""
    env = EvacuationEnv(**env_kwargs)
    L, W = env.width, env.height
    G = (L + 2, W + 2)
    floor = np.array(env.map.space, dtype=np.float64)
    valid = np.zeros(G, np.uint8)
    exitm = np.zeros(G, np.uint8)
    for x in range(G[0]):
        for y in range(G[1]):
            valid[x, y] = env.map.Check_Valid(x, y)
            exitm[x, y] = env.map.checkSavefy((x + 0.5, y + 0.5))
    barrier = np.zeros(G, np.uint8)
    for (bx, by) in env.map.barrier_list:
        barrier[bx, by] = 1
    ox0, oy0 = -OBS_PAD, -OBS_PAD
    OX, OY = G[0] + 2 * OBS_PAD, G[1] + 2 * OBS_PAD
    pm = env.map.fire_model
    om = env.fire_model
    assert pm.progressive_model.current_step == 0
    dp = np.zeros((t_max + 1,) + G, np.float64)
    do = np.zeros((t_max + 1, OX, OY), np.float64)
    for t in range(t_max + 1):
        for x in range(G[0]):
            for y in range(G[1]):
                dp[t, x, y] = pm.get_max_danger((x + 0.5, y + 0.5))
        for i in range(OX):
            for j in range(OY):
                do[t, i, j] = om.get_max_danger((ox0 + i, oy0 + j))
        pm.update()
        om.update()
    # danger at integer coordinates of the map's model at t = 0 (Init_Potential input)
    fm0 = FireSpreadModel([FireSource(center=((A[0] + B[0]) / 2, (A[1] + B[1]) / 2), size=(2, 2))
                           for (A, B) in env.map.Barrier])
    d0 = np.array([[fm0.get_max_danger((x, y)) for y in range(G[1])] for x in range(G[0])])
    return dict(L=np.int32(L), W=np.int32(W), floor=floor, valid=valid, exit_mask=exitm,
                barrier=barrier, danger_p=dp, danger_o=do, obs_origin=np.array([ox0, oy0], np.int32),
                danger_int0=d0, exit=np.array(env.exit_location, np.int32),
                robot_range=np.array(env.map.robot_range, np.int32))


# ----------------------------------------------------------------------------
# trajectories
# ----------------------------------------------------------------------------

def run_traj(make_env, n_robots, seed, episodes, max_steps_total, full=True, act_seed=None):
    random.seed(seed)
    np.random.seed(seed)
    env = make_env()
    act_rng = np.random.RandomState(1000 + seed if act_seed is None else act_seed)
    rec = {k: [] for k in ["rng_py", "rng_np", "reward", "done", "is_reset", "actions",
                           "fire_step", "time", "cur_step", "evac", "dead"]}
    snaps = {k: [] for k in FIELDS}
    digs = {k: [] for k in FIELDS}
    total = 0
    for ep in range(episodes):
        py, npk = rng_states()
        obs = env.reset()
        obs = np.array(obs, dtype=np.float64)
        rec["rng_py"].append(py); rec["rng_np"].append(npk)
        _record(env, obs, rec, snaps, digs, full, reward=0.0, done=False, reset=True,
                actions=np.full(n_robots, -1, np.int32))
        done = False
        while not done and total < max_steps_total:
            a = act_rng.randint(0, 5, size=n_robots).astype(np.int32)
            py, npk = rng_states()
            rec["rng_py"].append(py); rec["rng_np"].append(npk)
            if n_robots == 1 and not isinstance(env, EvacuationEnvMulti):
                obs, r, done, info = env.step(int(a[0]))
            else:
                obs, r, done, info = env.step([int(v) for v in a])
            total += 1
            _record(env, np.array(obs, dtype=np.float64), rec, snaps, digs, full, reward=r,
                    done=done, reset=False, actions=a)
        if total >= max_steps_total:
            break
    out = {k: np.array(v) for k, v in rec.items()}
    for k in FIELDS:
        out["dig_" + k] = np.array(digs[k])
        if full:
            out["snap_" + k] = np.array(snaps[k])
    py, npk = rng_states()
    out["rng_py_final"] = py
    out["rng_np_final"] = npk
    return out


def _record(env, obs, rec, snaps, digs, full, reward, done, reset, actions):
    st = env_state(env)
    st["obs"] = obs.reshape(-1, 11, 11, 6)
    for k in FIELDS:
        digs[k].append(digest(k, st[k]))
        if full:
            snaps[k].append(np.asarray(st[k]))
    assert isinstance(reward, float), type(reward)
    rec["reward"].append(np.float64(reward))
    rec["done"].append(bool(done))
    rec["is_reset"].append(bool(reset))
    rec["actions"].append(actions)
    rec["fire_step"].append(st["fire_step"])
    rec["time"].append(st["time"])
    rec["cur_step"].append(st["cur_step"])
    rec["evac"].append(int((st["flags"] & 1).sum()))
    rec["dead"].append(int(((st["flags"] >> 1) & 1).sum()))


# ----------------------------------------------------------------------------
# RNG recipe vectors (Appendix B of SURVEY.md)
# ----------------------------------------------------------------------------

def rng_vectors():
    out = {}
    random.seed(12345)
    out["py_state0"] = rng_states()[0]
    out["py_random"] = np.array([random.random() for _ in range(64)])
    out["py_state1"] = rng_states()[0]
    out["py_uniform"] = np.array([random.uniform(-0.1, 0.1) for _ in range(64)])
    out["py_state2"] = rng_states()[0]
    ns = [1, 2, 3, 5, 7, 34, 100, 126, 1000, 65535]
    out["randbelow_n"] = np.array(ns * 8, np.int64)
    out["py_randbelow"] = np.array([random._inst._randbelow(n) if hasattr(random, "_inst") else random.randrange(n)
                                    for n in ns * 8], np.int64)
    out["py_state3"] = rng_states()[0]
    lst = list(range(7))
    random.shuffle(lst)
    out["py_shuffle7"] = np.array(lst)
    out["py_state4"] = rng_states()[0]
    np.random.seed(777)
    out["np_state0"] = rng_states()[1]
    out["np_uniform"] = np.array([np.random.uniform(0.8, 2.0) for _ in range(64)])
    out["np_random"] = np.array([np.random.random() for _ in range(16)])
    out["np_state1"] = rng_states()[1]
    # seeding: Python random.seed(int) and numpy RandomState(int)
    for s in [0, 1, 1234, 99999, 2**31 + 5]:
        random.seed(s)
        out[f"py_seed_{s}"] = rng_states()[0]
        np.random.seed(s % 2**32)
        out[f"np_seed_{s}"] = rng_states()[1]
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    cfg1 = dict(width=36, height=30, fire_zones=[[18, 14], [19, 14], [18, 15], [19, 15], [18, 16], [19, 16]],
                exit_location=[36, 15], num_people=150)

    print("rng vectors")
    np.savez_compressed(os.path.join(OUT, "rng_vectors.npz"), **rng_vectors())

    print("cfg1 layout")
    lay = layout_tables(cfg1, 180)
    np.savez_compressed(os.path.join(OUT, "cfg1_layout.npz"), **lay)

    print("cfg1 single trajectory")
    tr = run_traj(lambda: EvacuationEnv(**cfg1), 1, seed=0, episodes=3, max_steps_total=400, full=True)
    np.savez_compressed(os.path.join(OUT, "cfg1_single_traj.npz"), **tr)
    print("  steps", len(tr["reward"]), "resets", tr["is_reset"].sum())

    print("cfg1 multi trajectory")
    tr = run_traj(lambda: EvacuationEnvMulti(**cfg1), 2, seed=1, episodes=2, max_steps_total=300, full=True)
    np.savez_compressed(os.path.join(OUT, "cfg1_multi_traj.npz"), **tr)
    print("  steps", len(tr["reward"]), "resets", tr["is_reset"].sum())

    # scaled rows: the reference code at larger sizes (its hard-coded barrier,
    # fire centres and robot x-range stay; SURVEY.md §6 caveat)
    for tag, L, W, P, R, T in [("g64", 64, 64, 569, 8, 30), ("g128", 128, 128, 2276, 16, 24)]:
        kw = dict(width=L, height=W, fire_zones=None, exit_location=[L, W // 2], num_people=P)
        print(tag, "layout")
        lay = layout_tables(kw, T + 2)
        np.savez_compressed(os.path.join(OUT, f"{tag}_layout.npz"), **lay)
        init = [[15 + (i * 15) // max(R - 1, 1), 4 + (i * (W - 8)) // max(R - 1, 1)] for i in range(R)]
        print(tag, "trajectory", init)
        tr = run_traj(lambda: EvacuationEnvMultiR(init, **kw), R, seed=2, episodes=1, max_steps_total=T,
                      full=False)
        tr["robot_init"] = np.array(init, np.int32)
        np.savez_compressed(os.path.join(OUT, f"{tag}_multi_traj.npz"), **tr)
        print("  steps", len(tr["reward"]))


if __name__ == "__main__":
    main()
