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
    if name in ("cfg1_single_traj", "cfg1_dropin_single"):
        return "cfg1_layout", 150, lay.reference_single()
    if name in ("cfg1_multi_traj", "cfg1_dropin_multi"):
        return "cfg1_layout", 150, lay.reference_multi()
    if name == "g64_multi_traj":
        return "g64_layout", 569, lay.reference_scaled_multi(64, 64, 8)
    if name in ("g128_multi_traj", "g128_long_traj"):
        return "g128_layout", 2276, lay.reference_scaled_multi(128, 128, 16)
    raise KeyError(name)


# trajectories that run past the fire steps of their committed layout tables use the host
# builder's tables, pinned for every fire step by g128_danger_digests.npz
# (tests/test_oracle_golden.py::test_g128_danger_tables_all_fire_steps)
BUILT_TABLES = {"g128_long_traj"}


def traj_tables(name):
    """(LayoutTables, P) of a trajectory fixture: the committed reference tables, or the host
    builder's (full fire schedule) for BUILT_TABLES."""
    from evacx.layout import LayoutTables, build_tables
    lname, P, spec = traj_spec(name)
    if name in BUILT_TABLES:
        return build_tables(spec, t_max=180), P
    t = load(lname)
    return LayoutTables(spec=spec, floor=t["floor"], valid=t["valid"], exit_mask=t["exit_mask"],
                        barrier=t["barrier"], danger_p=t["danger_p"], danger_o=t["danger_o"],
                        obs_origin=tuple(int(v) for v in t["obs_origin"])), P


def oracle_layout(traj_name):
    """Oracle layout built from the committed reference tables of a trajectory fixture."""
    from oracle.oracle import Layout
    lname, P, spec = traj_spec(traj_name)
    t = load(lname)
    if traj_name in BUILT_TABLES:
        tb, _ = traj_tables(traj_name)
        t = dict(floor=tb.floor, valid=tb.valid, exit_mask=tb.exit_mask, barrier=tb.barrier,
                 danger_p=tb.danger_p, danger_o=tb.danger_o, obs_origin=np.asarray(tb.obs_origin))
    return Layout(L=spec.L, W=spec.W, P=P, R=spec.R, floor=t["floor"], valid=t["valid"],
                  exit_mask=t["exit_mask"], barrier=t["barrier"], danger_p=t["danger_p"],
                  danger_o=t["danger_o"], obs_origin=t["obs_origin"], exit=spec.exit,
                  robot_range=spec.robot_range, reset_view=spec.reset_view,
                  reset_robots=spec.reset_robots, robot_init=spec.robot_init), spec, t


def state_fields(st, obs):
    return dict(pos=st["pos"], health=st["health"], acc=st["acc"], flags=st["flags"], rmap=st["rmap"],
                thmap=st["thmap"], robots=st["robots"], view=st["view"], obs=obs)


# ----------------------------------------------------------------------------
# learner fixtures (tools/capture_golden.py dqn_fixtures)
# ----------------------------------------------------------------------------
def fmix32(h):
    h = np.asarray(h, np.uint64) & 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def closed_form_params(shapes, salt=0):
    """Closed-form deterministic parameters, no torch RNG: tensor t of the state_dict
    (ordered name -> shape) gets w[k] = bound * (2 u - 1), u = fmix32(k ^ hash(t, salt)) / 2^32,
    bound = 1 / sqrt(fan_in) (nn.Linear / nn.Conv2d default init range). The weights and
    biases of one layer share the weight's fan-in."""
    out = {}
    fan = None
    for t, (name, shape) in enumerate(shapes.items()):
        n = int(np.prod(shape))
        if name.endswith(".weight"):
            fan = int(np.prod(shape[1:]))
        key = int(fmix32(np.uint64((t + 1) * 0x9E3779B1 + salt * 0x7F4A7C15)))
        u = fmix32(np.arange(n, dtype=np.uint64) ^ np.uint64(key)).astype(np.float64) / 2.0 ** 32
        out[name] = ((2.0 * u - 1.0) / np.sqrt(fan)).astype(np.float32).reshape(shape)
    return out


def mlp_shapes(hidden=512, in_dim=726, actions=5):
    return {"fc1.weight": (hidden, in_dim), "fc1.bias": (hidden,), "fc2.weight": (hidden // 2, hidden),
            "fc2.bias": (hidden // 2,), "fc3.weight": (actions, hidden // 2), "fc3.bias": (actions,)}


def conv_shapes(hidden=512, actions=5):
    return {"conv1.weight": (32, 6, 3, 3), "conv1.bias": (32,), "conv2.weight": (64, 32, 3, 3), "conv2.bias": (64,),
            "conv3.weight": (128, 64, 3, 3), "conv3.bias": (128,), "fc1.weight": (hidden, 15488), "fc1.bias": (hidden,),
            "fc2.weight": (hidden // 2, hidden), "fc2.bias": (hidden // 2,), "fc3.weight": (actions, hidden // 2),
            "fc3.bias": (actions,)}


SEL_FULL = 16384  # tensors up to this size are stored whole, larger ones at SEL_N fixed positions
SEL_N = 2048


def select_positions(n, t):
    """Fixed positions at which a large tensor is stored (sorted, deterministic per tensor index)."""
    if n <= SEL_FULL:
        return np.arange(n)
    return np.sort(np.random.RandomState(1000 + t).choice(n, SEL_N, replace=False))
