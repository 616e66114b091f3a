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
  (``agents/dqn_agent.py:15-168``) for deterministic, closed-form weights
  (``dqn_forward.npz``, ``dqn_learn.npz``; ``dqn_fixtures``): observations made by the
  reference's own ``EvacuationEnv._get_state`` (``envs/evacuation_env.py:84-120``),
  Q-values of the full-size conv network and of the MLP variant, and three ``learn``
  steps of each with the sampled batch indices, the dropout masks (forward hooks on
  the ``Dropout`` modules), the loss, the total gradient norm, the gradients and the
  parameters / Adam moments after every step,
* the QMIX mixer's learn step with the reference's own ``MixingNetwork``
  (``runners/train_qmix.py:39-113``; ``qmix_mixer.npz``, ``qmix_fixtures``),
* a long 128x128 R16 trajectory (``g128_long_traj.npz``: past the fire's last step,
  with a reset) and the per-step digests of the 128x128 danger tables for all 181
  fire steps (``g128_danger_digests.npz``).

Usage:  PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tools/capture_golden.py [part ...]
  parts: base (the round-1 fixtures), dqn, g128long, g128danger, dropin, ckpt, qmix; default: all
"""
import hashlib
import os
import random
import sys

import numpy as np

REF = os.environ.get("EVX_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
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

def run_traj(make_env, n_robots, seed, episodes, max_steps_total, full=True, act_seed=None, episode_cap=None):
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
        ep_steps = 0
        while not done and total < max_steps_total and (episode_cap is None or ep_steps < episode_cap):
            ep_steps += 1
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


CFG1 = dict(width=36, height=30, fire_zones=[[18, 14], [19, 14], [18, 15], [19, 15], [18, 16], [19, 16]],
            exit_location=[36, 15], num_people=150)


# ----------------------------------------------------------------------------
# learner fixtures
# ----------------------------------------------------------------------------

def reference_observations(n, seed):
    """n observations made by the reference's EvacuationEnv._get_state on the cfg1 layout:
    window centres anywhere in the padded grid, People.rmap random bits, fire steps 0, 40,
    90 and 180 (the env's fire model advanced with its own update()). Also returns each
    one's compact form (occupancy bits of the 121 window cells where Check_Valid, centre,
    fire step) -- the evx_obs the build's fused kernels read."""
    rs = np.random.RandomState(seed)
    random.seed(seed)
    np.random.seed(seed)
    env = EvacuationEnv(**CFG1)
    L, W = env.width, env.height
    obs, comp = [], []
    steps = [0, 40, 90, 180]
    per = [n // 4 + (1 if i < n % 4 else 0) for i in range(4)]
    for t, k in zip(steps, per):
        while env.fire_model.progressive_model.current_step < t:
            env.fire_model.update()
        for _ in range(k):
            cx, cy = int(rs.randint(0, L + 2)), int(rs.randint(0, W + 2))
            rm = (rs.random_sample((L + 2, W + 2)) < rs.uniform(0.05, 0.6)).astype(np.float64)
            env.people.rmap = rm
            env.map.robot_position = [cx, cy]
            o = np.array(env._get_state(), dtype=np.float64)
            occ = np.zeros(4, np.uint32)
            for i in range(11):
                for j in range(11):
                    x, y = cx + i - 5, cy + j - 5
                    if env.map.Check_Valid(x, y) and rm[x][y] == 1:
                        c = i * 11 + j
                        occ[c >> 5] |= np.uint32(1 << (c & 31))
            obs.append(o)
            comp.append(np.concatenate([occ.view(np.int32), np.array([cx, cy, t, 0], np.int32)]))
    return np.stack(obs), np.stack(comp).astype(np.int32)


def _store(prefix, tensors, out):
    """Tensors by name at golden_util.select_positions (whole when small) + each one's
    float64 sum of squares."""
    from golden_util import select_positions
    for t, (name, v) in enumerate(tensors.items()):
        a = np.asarray(v, np.float32).reshape(-1)
        sel = select_positions(a.size, t)
        out[f"{prefix}{name}"] = a[sel]
        out[f"{prefix}{name}__ss"] = np.float64(np.sum(a.astype(np.float64) ** 2))


def dqn_fixtures():
    """DQNNetwork forward and DQNAgent.learn vectors (agents/dqn_agent.py:15-168)."""
    import torch
    import torch.nn as nn
    import torch.nn.functional as F
    from Louvre_Evacuation.agents import dqn_agent as ref_agent
    from golden_util import closed_form_params, conv_shapes, mlp_shapes

    torch.set_num_threads(8)

    class MLPNet(nn.Module):
        """The build's MLP variant of DQNNetwork: DQNNetwork's fc stack on the
        flattened (11, 11, 6) observation -- fc1 726->512, ReLU, Dropout(0.2), fc2, ReLU, fc3.
        Harness only: the learn() these fixtures record is the reference's own."""

        def __init__(self, hidden=512):
            super().__init__()
            self.fc1 = nn.Linear(726, hidden)
            self.fc2 = nn.Linear(hidden, hidden // 2)
            self.fc3 = nn.Linear(hidden // 2, 5)
            self.dropout = nn.Dropout(0.2)

        def forward(self, x):
            x = x.reshape(x.shape[0], -1)
            x = self.dropout(F.relu(self.fc1(x)))
            return self.fc3(F.relu(self.fc2(x)))

    def load(net, params):
        net.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in params.items()})

    masks = []

    def hook(_m, inp, outp):
        masks.append((outp[0] if isinstance(outp, tuple) else outp).detach().ne(0).numpy().copy())

    obs, comp = reference_observations(160, seed=11)
    out = {"obs": obs.astype(np.float32), "obs_compact": comp}

    # ---------------- forward: full-size networks, closed-form weights
    fw = {}
    x = torch.from_numpy(obs[:16].astype(np.float32))
    for kind, net, shapes in [("conv", ref_agent.DQNNetwork((11, 11, 6), 5), conv_shapes()),
                              ("mlp", MLPNet(), mlp_shapes())]:
        load(net, closed_form_params(shapes, salt=1))
        net.eval()
        with torch.no_grad():
            fw[f"{kind}_q_eval"] = net(x).numpy()
        net.train()
        h = net.dropout.register_forward_hook(hook)
        masks.clear()
        torch.manual_seed(5)
        with torch.no_grad():
            fw[f"{kind}_q_train"] = net(x).numpy()
        h.remove()
        fw[f"{kind}_mask_train"] = masks[0].astype(np.uint8)
    fw["obs_idx"] = np.arange(16)
    np.savez_compressed(os.path.join(OUT, "dqn_forward.npz"), **fw)
    print("  dqn forward", {k: v.shape for k, v in fw.items()})

    # ---------------- learn: 3 steps of the reference's DQNAgent.learn
    lo = dict(out)  # the observations (f32, as DQNAgent.learn's FloatTensor) and their compact forms
    cfg = dict(gamma=0.99, epsilon=1.0, epsilon_min=0.02, epsilon_decay=0.9995, learning_rate=1e-4,
               batch_size=32, warmup_steps=0, memory_size=50000)
    orig_sample, orig_clip = random.sample, torch.nn.utils.clip_grad_norm_
    for kind, mk, shapes in [("conv32", lambda: ref_agent.DQNNetwork((11, 11, 6), 5, hidden_size=32),
                              conv_shapes(hidden=32)),
                             ("mlp", MLPNet, mlp_shapes())]:
        random.seed(21)
        np.random.seed(21)
        torch.manual_seed(21)
        agent = ref_agent.DQNAgent((11, 11, 6), 5, torch.device("cpu"), cfg)
        agent.q_network, agent.target_network = mk(), mk()
        p0 = closed_form_params(shapes, salt=2)
        load(agent.q_network, p0)
        agent.update_target_network()
        agent.optimizer = torch.optim.Adam(agent.q_network.parameters(), lr=cfg["learning_rate"])
        rs = np.random.RandomState(31)
        NM = 48
        idx_s, idx_s2 = rs.permutation(NM), NM + rs.permutation(NM)
        acts = rs.randint(0, 5, NM)
        rews = np.round(rs.normal(0.0, 30.0, NM), 3)
        dones = rs.random_sample(NM) < 0.25
        for i in range(NM):
            agent.remember(obs[idx_s[i]], int(acts[i]), float(rews[i]), obs[idx_s2[i]], bool(dones[i]))
        lo[f"{kind}_mem_s"], lo[f"{kind}_mem_s2"] = idx_s, idx_s2
        lo[f"{kind}_mem_a"], lo[f"{kind}_mem_r"], lo[f"{kind}_mem_done"] = acts, rews, dones
        mem_ids = {id(t): i for i, t in enumerate(agent.memory)}
        rec = {}

        def rec_sample(pop, k):
            r = orig_sample(pop, k)
            rec["idx"] = np.array([mem_ids[id(t)] for t in r], np.int32)
            return r

        def rec_clip(params, max_norm, *a, **kw):
            params = list(params)
            rec["grads"] = {n: p.grad.detach().numpy().copy() for n, p in agent.q_network.named_parameters()}
            nrm = orig_clip(params, max_norm, *a, **kw)
            rec["norm"] = float(nrm)
            return nrm

        hq = agent.q_network.dropout.register_forward_hook(hook)
        ht = agent.target_network.dropout.register_forward_hook(hook)
        random.sample, torch.nn.utils.clip_grad_norm_ = rec_sample, rec_clip
        try:
            for step in range(3):
                masks.clear()
                loss = agent.learn()
                assert len(masks) == 2, len(masks)
                lo[f"{kind}_s{step}_idx"] = rec["idx"]
                lo[f"{kind}_s{step}_mask_online"] = masks[0].astype(np.uint8)
                lo[f"{kind}_s{step}_mask_target"] = masks[1].astype(np.uint8)
                lo[f"{kind}_s{step}_loss"] = np.float64(loss)
                lo[f"{kind}_s{step}_norm"] = np.float64(rec["norm"])
                lo[f"{kind}_s{step}_epsilon"] = np.float64(agent.epsilon)
                _store(f"{kind}_s{step}_grad_", rec["grads"], lo)
                _store(f"{kind}_s{step}_param_", {n: p.detach().numpy() for n, p in
                                                  agent.q_network.named_parameters()}, lo)
                st = agent.optimizer.state
                _store(f"{kind}_s{step}_m_", {n: st[p]["exp_avg"].numpy() for n, p in
                                              agent.q_network.named_parameters()}, lo)
                _store(f"{kind}_s{step}_v_", {n: st[p]["exp_avg_sq"].numpy() for n, p in
                                              agent.q_network.named_parameters()}, lo)
        finally:
            random.sample, torch.nn.utils.clip_grad_norm_ = orig_sample, orig_clip
            hq.remove()
            ht.remove()
        print("  dqn learn", kind, [float(lo[f"{kind}_s{s}_loss"]) for s in range(3)])
    np.savez_compressed(os.path.join(OUT, "dqn_learn.npz"), **lo)


def g128_long():
    """128x128 R16 trajectory past the fire's last step (180) with a reset at step 230
    (an episode cap, as the runners' `while steps < max_steps` loop does)."""
    L = W = 128
    R, P = 16, 2276
    kw = dict(width=L, height=W, fire_zones=None, exit_location=[L, W // 2], num_people=P)
    init = [[15 + (i * 15) // max(R - 1, 1), 4 + (i * (W - 8)) // max(R - 1, 1)] for i in range(R)]
    tr = run_traj(lambda: EvacuationEnvMultiR(init, **kw), R, seed=3, episodes=2, max_steps_total=260,
                  full=False, episode_cap=230)
    tr["robot_init"] = np.array(init, np.int32)
    np.savez_compressed(os.path.join(OUT, "g128_long_traj.npz"), **tr)
    print("  steps", len(tr["reward"]), "resets", int(tr["is_reset"].sum()))


def g128_danger():
    """sha256 per fire step (0..180) of the 128x128 danger tables (layout_tables' danger_p /
    danger_o, float64 bytes): pins every step, where g128_layout.npz holds the first 27."""
    L = W = 128
    kw = dict(width=L, height=W, fire_zones=None, exit_location=[L, W // 2], num_people=2276)
    lay = layout_tables(kw, 180)
    dp = np.stack([np.frombuffer(hashlib.sha256(np.ascontiguousarray(lay["danger_p"][t]).tobytes()).digest(),
                                 np.uint8) for t in range(181)])
    do = np.stack([np.frombuffer(hashlib.sha256(np.ascontiguousarray(lay["danger_o"][t]).tobytes()).digest(),
                                 np.uint8) for t in range(181)])
    np.savez_compressed(os.path.join(OUT, "g128_danger_digests.npz"), danger_p=dp, danger_o=do,
                        danger_p_max=lay["danger_p"].max(axis=(1, 2)), danger_o_sum=lay["danger_o"].sum(axis=(1, 2)))


def _traj_arrays(ppl):
    """Person.trajectory lists flattened: kind 0 = {'pos','step'} entry, 1 = record_position
    entry ({'pos','health','savety','dead'}); offsets per person."""
    kind, xy, step, health, flags, off = [], [], [], [], [], [0]
    for p in ppl:
        for e in p.trajectory:
            xy.append(e["pos"])
            if "step" in e:
                kind.append(0); step.append(e["step"]); health.append(np.nan); flags.append(0)
            else:
                kind.append(1); step.append(-1); health.append(float(e["health"]))
                flags.append((1 if e["savety"] else 0) | (2 if e["dead"] else 0))
        off.append(len(kind))
    return dict(traj_kind=np.array(kind, np.int8), traj_pos=np.array(xy, np.float64),
                traj_step=np.array(step, np.int32), traj_health=np.array(health, np.float64),
                traj_flags=np.array(flags, np.uint8), traj_off=np.array(off, np.int64))


# action kinds of the drop-in fixture: code -> the Python object handed to env.step
DROPIN_ACTIONS = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: None, 6: 3.0, 7: "f64_1", 8: True, 9: 7, 10: 2.5, 11: "arr_4"}


def dropin_action(code):
    v = DROPIN_ACTIONS[int(code)]
    return np.float64(1) if v == "f64_1" else np.array(4) if v == "arr_4" else v


def dropin_extras(multi, seed, episodes):
    """EvacuationEnv / EvacuationEnvMulti driven with patrol (None), float, bool, 0-d array and
    out-of-range actions (envs/map.py:172-197), random.gauss draws between steps (so the
    cached gauss_next must survive env steps), per-step robot positions and digests, and every
    person's trajectory at the end of each episode (envs/people.py:52-59,306,
    envs/evacuation_env.py:79-80,134-135)."""
    cfg1 = dict(width=36, height=30, fire_zones=None, exit_location=[36, 15], num_people=150)
    random.seed(seed)
    np.random.seed(seed)
    env = EvacuationEnvMulti(**cfg1) if multi else EvacuationEnv(**cfg1)
    R = 2 if multi else 1
    arng = np.random.RandomState(500 + seed)
    rec = {k: [] for k in ["codes", "reward", "done", "is_reset", "robots", "view", "gauss", "rng_py", "rng_np",
                           "dig_pos", "dig_health", "dig_obs"]}
    trajs = []
    for ep in range(episodes):
        py, npk = rng_states()
        rec["rng_py"].append(py); rec["rng_np"].append(npk)
        obs = env.reset()
        codes = np.full(R, -1, np.int32)
        r, done, k = 0.0, False, 0
        while True:
            st = env_state(env)
            rec["codes"].append(codes); rec["reward"].append(np.float64(r)); rec["done"].append(bool(done))
            rec["is_reset"].append(k == 0); rec["robots"].append(st["robots"]); rec["view"].append(st["view"])
            rec["dig_pos"].append(digest("pos", st["pos"])); rec["dig_health"].append(digest("health", st["health"]))
            rec["dig_obs"].append(digest("obs", np.array(obs, np.float64).reshape(-1, 11, 11, 6)))
            # a gauss draw every 3rd step leaves a cached second variate in the stream
            rec["gauss"].append(random.gauss(0.0, 1.0) if k % 3 == 1 else np.nan)
            if done or k >= 400:
                break
            # the first step patrols every robot (sets map.robot_direction, envs/map.py:174-177)
            codes = (np.full(R, 5, np.int32) if k == 0 else arng.choice(
                [0, 1, 2, 3, 4, 5, 5, 5, 6, 7, 8, 9, 10, 11], size=R).astype(np.int32))
            acts = [dropin_action(c) for c in codes]
            if k > 0:
                py, npk = rng_states()
                rec["rng_py"].append(py); rec["rng_np"].append(npk)
            obs, r, done, info = env.step(acts if multi else acts[0])
            k += 1
        rec["rng_py"].append(rng_states()[0]); rec["rng_np"].append(rng_states()[1])
        trajs.append(_traj_arrays(env.people.list))
    out = {k: np.array(v) for k, v in rec.items() if k not in ("rng_py", "rng_np")}
    out["rng_py_final"], out["rng_np_final"] = rng_states()
    for i, t in enumerate(trajs):
        for k, v in t.items():
            out[f"ep{i}_{k}"] = v
    out["robot_traj"] = np.array([[*p, s] for p, s in env.robot_trajectory], np.float64)
    return out


def ref_checkpoint():
    """A checkpoint written by the reference's own DQNAgent.save (agents/dqn_agent.py:174-182)
    after two DQNAgent.learn steps, so the optimizer state holds Adam moments. The network is
    the reference's DQNNetwork at hidden_size 2 (the constructor default patched in this
    process only) so the fixture stays ~2 MB; its eval-mode Q-values on 8 reference
    observations are recorded beside it. The file is committed gzip'd byte for byte."""
    import gzip
    import torch
    from Louvre_Evacuation.agents import dqn_agent as ref_agent

    torch.set_num_threads(8)
    init = ref_agent.DQNNetwork.__init__
    init.__defaults__ = (2,)
    try:
        random.seed(21)
        np.random.seed(21)
        torch.manual_seed(21)
        agent = ref_agent.DQNAgent((11, 11, 6), 5, torch.device("cpu"),
                                   {"batch_size": 8, "warmup_steps": 0, "epsilon": 0.5, "memory_size": 100})
        obs, _ = reference_observations(24, seed=31)
        obs = obs.astype(np.float32)
        for i in range(16):
            agent.remember(obs[i], i % 5, float(i) * 0.25 - 1.0, obs[i + 1], i % 7 == 6)
        losses = [agent.learn() for _ in range(2)]
        path = os.path.join(OUT, "ref_ckpt_h2.pt")
        agent.save(path)
        raw = open(path, "rb").read()
        os.remove(path)
        with gzip.open(path + ".gz", "wb", compresslevel=9) as f:
            f.write(raw)
        agent.q_network.eval()
        with torch.no_grad():
            q = agent.q_network(torch.from_numpy(obs[16:24])).numpy()
        np.savez_compressed(os.path.join(OUT, "ref_ckpt_h2_q.npz"), obs=obs[16:24], q_eval=q,
                            losses=np.array(losses, np.float64), epsilon=np.float64(agent.epsilon),
                            steps=np.int64(agent.steps))
        print("  checkpoint bytes", len(raw), "losses", losses)
    finally:
        init.__defaults__ = (512,)


def reference_mixing_class():
    """The reference's MixingNetwork. It is defined inside train_qmix()
    (runners/train_qmix.py:39-54), so it cannot be imported: its class statement is taken out
    of the file's syntax tree and executed here -- the reference's own code, run in this
    container; nothing of it is written out."""
    import ast
    import torch
    path = os.path.join(REF, "Louvre_Evacuation", "runners", "train_qmix.py")
    tree = ast.parse(open(path, encoding="utf-8").read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "train_qmix")
    cls = next(n for n in ast.walk(fn) if isinstance(n, ast.ClassDef) and n.name == "MixingNetwork")
    ns = {"torch": torch}
    exec(compile(ast.Module(body=[cls], type_ignores=[]), path, "exec"), ns)
    return ns["MixingNetwork"]


def qmix_fixtures():
    """The mixer side of three QMIX learn steps (runners/train_qmix.py:78-113) with the
    reference's own MixingNetwork (n_agents = 2, embed 32, torch.randn init under a fixed seed,
    target mixer loaded from the online one as at :57-58), Adam(lr = 1e-3): the agents' chosen
    Q-values and target max-Q values are the step's inputs (leaf tensors in place of
    agent{1,2}.q_network(...).gather / target_network(...).max, which dqn_learn.npz pins), then
    the reference's exact sequence -- stack, mixing, target_mixing under no_grad, y_tot =
    r + gamma * Q_tot' * ~done, mse_loss, zero_grad, backward, clip_grad_norm_(mixing, 1.0),
    step. Recorded per step: inputs, loss, d loss / d q (what flows into each agent's
    backward), the mixer's raw and clipped gradients, its total norm, parameters and Adam
    moments after the step. Batch 32 (configs/dqn.yaml batch_size), gamma 0.99."""
    import torch
    MixingNetwork = reference_mixing_class()
    torch.manual_seed(5)
    mixing = MixingNetwork(n_agents=2)
    target_mixing = MixingNetwork(n_agents=2)
    target_mixing.load_state_dict(mixing.state_dict())
    mix_optimizer = torch.optim.Adam(mixing.parameters(), lr=1e-3)
    out = {f"init_{k}": v.detach().numpy().copy() for k, v in mixing.state_dict().items()}
    out["names"] = np.array(list(mixing.state_dict().keys()))
    g = torch.Generator().manual_seed(7)
    B, gamma = 32, 0.99
    for step in range(3):
        q = (torch.randn(B, 2, generator=g) * 6.0 + 1.0).requires_grad_(True)
        tq = torch.randn(B, 2, generator=g) * 6.0 + 1.0
        r_b = torch.randn(B, generator=g) * 20.0
        d_b = torch.rand(B, generator=g) < 0.15
        q1, q2 = q[:, 0], q[:, 1]
        q_cat = torch.stack([q1, q2], dim=1)
        q_tot = mixing(q_cat)
        with torch.no_grad():
            target_q_cat = torch.stack([tq[:, 0], tq[:, 1]], dim=1)
            target_q_tot = target_mixing(target_q_cat)
            y_tot = r_b + gamma * target_q_tot * (~d_b)
        loss = torch.nn.functional.mse_loss(q_tot, y_tot)
        mix_optimizer.zero_grad()
        loss.backward()
        raw = {k: p.grad.detach().clone() for k, p in mixing.named_parameters()}
        norm = torch.nn.utils.clip_grad_norm_(mixing.parameters(), 1.0)
        mix_optimizer.step()
        pre = f"s{step}_"
        out[pre + "q"] = q.detach().numpy().copy()
        out[pre + "tq"] = tq.numpy().copy()
        out[pre + "r"] = r_b.numpy().copy()
        out[pre + "d"] = d_b.numpy().astype(np.uint8)
        out[pre + "loss"] = np.float32(loss.item())
        out[pre + "dq"] = q.grad.detach().numpy().copy()
        out[pre + "norm"] = np.float32(norm.item())
        out[pre + "hidden_active"] = ((q_cat.detach() @ mixing.fc1_weight.detach().abs()) > 0).numpy()
        for k, p in mixing.named_parameters():
            st = mix_optimizer.state[p]
            out[pre + "raw_" + k] = raw[k].numpy()
            out[pre + "grad_" + k] = p.grad.detach().numpy().copy()
            out[pre + "param_" + k] = p.detach().numpy().copy()
            out[pre + "m_" + k] = st["exp_avg"].numpy().copy()
            out[pre + "v_" + k] = st["exp_avg_sq"].numpy().copy()
        print(f"  step {step}: loss {loss.item():.6g} norm {norm.item():.6g}")
    np.savez_compressed(os.path.join(OUT, "qmix_mixer.npz"), **out)


def main():
    os.makedirs(OUT, exist_ok=True)
    parts = sys.argv[1:] or ["base", "dqn", "g128long", "g128danger", "dropin", "ckpt", "qmix"]
    if "qmix" in parts:
        print("qmix mixer")
        qmix_fixtures()
    if "ckpt" in parts:
        print("reference checkpoint")
        ref_checkpoint()
    if "dropin" in parts:
        for multi, tag in [(False, "single"), (True, "multi")]:
            print("drop-in extras", tag)
            tr = dropin_extras(multi, seed=11 if multi else 10, episodes=2)
            np.savez_compressed(os.path.join(OUT, f"cfg1_dropin_{tag}.npz"), **tr)
            print("  steps", len(tr["reward"]))
    if "dqn" in parts:
        print("dqn fixtures")
        dqn_fixtures()
    if "g128danger" in parts:
        print("g128 danger digests")
        g128_danger()
    if "g128long" in parts:
        print("g128 long trajectory")
        g128_long()
    if "base" not in parts:
        return
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
