"""Shared helpers for golden-fixture tests (fixtures made by tools/capture_golden.py)."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PKG = os.path.join(ROOT, "dqn-marl_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

FIELDS = ["pos", "health", "acc", "flags", "rmap", "thmap", "robots", "view", "obs"]
DTYPES = {"pos": np.int32, "health": np.float64, "acc": np.float64, "flags": np.uint8, "rmap": np.uint8,
          "thmap": np.int32, "robots": np.int32, "view": np.int32, "obs": np.float64}

# fixture name -> (layout file, P, robot init, reset semantics)
CFG1 = dict(width=36, height=30, P=150)


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def digest(name, a):
    b = np.ascontiguousarray(np.asarray(a, dtype=DTYPES[name])).tobytes()
    return np.frombuffer(hashlib.sha256(b).digest(), dtype=np.uint8)


def traj_spec(name):
    """(layout fixture, P, LayoutSpec factory args) for each trajectory fixture."""
    from evacx import layout as lay
    if name == "cfg1_single_traj":
        return "cfg1_layout", 150, lay.reference_single()
    if name == "cfg1_multi_traj":
        return "cfg1_layout", 150, lay.reference_multi()
    if name == "g64_multi_traj":
        return "g64_layout", 569, lay.reference_scaled_multi(64, 64, 8)
    if name == "g128_multi_traj":
        return "g128_layout", 2276, lay.reference_scaled_multi(128, 128, 16)
    raise KeyError(name)


def oracle_layout(traj_name):
    """Oracle layout built from the committed reference tables of a trajectory fixture."""
    from oracle.oracle import Layout
    lname, P, spec = traj_spec(traj_name)
    t = load(lname)
    return Layout(L=spec.L, W=spec.W, P=P, R=spec.R, floor=t["floor"], valid=t["valid"],
                  exit_mask=t["exit_mask"], barrier=t["barrier"], danger_p=t["danger_p"],
                  danger_o=t["danger_o"], obs_origin=t["obs_origin"], exit=spec.exit,
                  robot_range=spec.robot_range, reset_view=spec.reset_view,
                  reset_robots=spec.reset_robots, robot_init=spec.robot_init), spec, t


def state_fields(st, obs):
    return dict(pos=st["pos"], health=st["health"], acc=st["acc"], flags=st["flags"], rmap=st["rmap"],
                thmap=st["thmap"], robots=st["robots"], view=st["view"], obs=obs)
