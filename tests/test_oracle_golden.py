"""Pin the CPU oracle (oracle/evac_oracle.c) and the host layout builder against
golden vectors captured from the reference (tools/capture_golden.py)."""
import numpy as np
import pytest

from golden_util import FIELDS, digest, load, oracle_layout, state_fields
from evacx import layout as lay
from oracle import oracle as orc


# ---------------------------------------------------------------- RNG recipes
def test_mt_random_uniform_randbelow_shuffle():
    v = load("rng_vectors")
    st = v["py_state0"].copy()
    out = np.array([orc.lib().orc_mt_random(orc._p(st)) for _ in range(64)])
    assert np.array_equal(out, v["py_random"])
    assert np.array_equal(st, v["py_state1"])
    u = np.array([-0.1 + (0.1 - -0.1) * orc.lib().orc_mt_random(orc._p(st)) for _ in range(64)])
    assert np.array_equal(u, v["py_uniform"])
    assert np.array_equal(st, v["py_state2"])
    rb = np.array([orc.lib().orc_mt_randbelow(orc._p(st), int(n)) for n in v["randbelow_n"]])
    assert np.array_equal(rb, v["py_randbelow"])
    assert np.array_equal(st, v["py_state3"])
    lst = list(range(7))
    for i in range(6, 0, -1):
        j = orc.lib().orc_mt_randbelow(orc._p(st), i + 1)
        lst[i], lst[j] = lst[j], lst[i]
    assert lst == list(v["py_shuffle7"])
    assert np.array_equal(st, v["py_state4"])
    ns = v["np_state0"].copy()
    nu = np.array([0.8 + (2.0 - 0.8) * orc.lib().orc_mt_random(orc._p(ns)) for _ in range(64)])
    assert np.array_equal(nu, v["np_uniform"])


@pytest.mark.parametrize("seed", [0, 1, 1234, 99999, 2**31 + 5])
def test_seeding(seed):
    v = load("rng_vectors")
    a = np.zeros(625, np.uint32)
    orc.lib().orc_seed_py(orc.C.c_uint32(seed), orc._p(a))
    assert np.array_equal(a, v[f"py_seed_{seed}"])
    orc.lib().orc_seed_np(orc.C.c_uint32(seed % 2**32), orc._p(a))
    assert np.array_equal(a, v[f"np_seed_{seed}"])


def test_pairwise_sum_matches_numpy():
    rng = np.random.RandomState(0)
    for n in [0, 1, 7, 8, 9, 127, 128, 129, 255, 1000, 2276, 9102]:
        a = rng.rand(n) * 30
        assert orc.pairwise_sum(a) == np.add.reduce(a), n


# ------------------------------------------------------------- layout tables
@pytest.mark.parametrize("lname,spec", [
    ("cfg1_layout", lay.reference_single()),
    ("g64_layout", lay.reference_scaled_multi(64, 64, 8)),
    ("g128_layout", lay.reference_scaled_multi(128, 128, 16)),
])
def test_layout_builder_matches_reference(lname, spec):
    g = load(lname)
    tb = lay.build_tables(spec, t_max=g["danger_p"].shape[0] - 1)
    for k in ["floor", "valid", "exit_mask", "barrier", "danger_p", "danger_o"]:
        assert np.array_equal(getattr(tb, k), g[k]), k
    assert tuple(tb.obs_origin) == tuple(g["obs_origin"])


def test_g128_danger_tables_all_fire_steps():
    """The host builder's 128x128 danger tables equal the reference's for EVERY fire step
    0..180 (sha256 of each step's float64 table, captured from the reference's
    FireSpreadModel.get_max_danger: envs/fire_model.py:138-188); g128_layout.npz holds the
    first 27 steps in full."""
    import hashlib
    d = load("g128_danger_digests")
    tb = lay.build_tables(lay.reference_scaled_multi(128, 128, 16), t_max=180)
    assert tb.danger_p.shape[0] == 181 and d["danger_p"].shape[0] == 181
    for t in range(181):
        dp = np.frombuffer(hashlib.sha256(np.ascontiguousarray(tb.danger_p[t]).tobytes()).digest(), np.uint8)
        do = np.frombuffer(hashlib.sha256(np.ascontiguousarray(tb.danger_o[t]).tobytes()).digest(), np.uint8)
        assert np.array_equal(dp, d["danger_p"][t]), t
        assert np.array_equal(do, d["danger_o"][t]), t


def test_known_answers_cfg1():
    g = load("cfg1_layout")
    fin = g["floor"][np.isfinite(g["floor"])]
    assert fin.max() == 41.99999999999998
    assert len(fin) == 1071
    assert g["barrier"].sum() == 145


# -------------------------------------------------------------- trajectories
def replay(traj_name, check_each):
    L, spec, _ = oracle_layout(traj_name)
    tr = load(traj_name)
    env = orc.Env(L)
    for k in range(len(tr["reward"])):
        if tr["is_reset"][k]:
            if k == 0:  # the recorded start state; later resets continue the streams
                env.py_mt[:] = tr["rng_py"][k]
                env.np_mt[:] = tr["rng_np"][k]
            assert np.array_equal(env.py_mt, tr["rng_py"][k]), k
            assert np.array_equal(env.np_mt, tr["rng_np"][k]), k
            obs, r, d = env.reset(), 0.0, False
        else:
            assert np.array_equal(env.py_mt, tr["rng_py"][k]), k
            assert np.array_equal(env.np_mt, tr["rng_np"][k]), k
            obs, r, d = env.step(tr["actions"][k])
        check_each(k, tr, env, obs, r, d)
    assert np.array_equal(env.py_mt, tr["rng_py_final"])
    assert np.array_equal(env.np_mt, tr["rng_np_final"])
    return tr


@pytest.mark.parametrize("traj", ["cfg1_single_traj", "cfg1_multi_traj", "g64_multi_traj", "g128_multi_traj",
                                  "g128_long_traj"])
def test_oracle_trajectory_bit_exact(traj):
    def check(k, tr, env, obs, r, d):
        st = state_fields(env.state(), obs)
        for f in FIELDS:
            assert np.array_equal(digest(f, st[f]), tr["dig_" + f][k]), (k, f)
        assert r == tr["reward"][k], k
        assert d == tr["done"][k], k
        assert env.fire_step == tr["fire_step"][k]
        assert env.scal[1] == tr["cur_step"][k] and float(env.time[0]) == tr["time"][k]
    tr = replay(traj, check)
    assert tr["is_reset"].sum() >= 1
    if traj == "g128_long_traj":  # past the fire's last step, and a reset at 128x128
        assert tr["fire_step"].max() == 180 and tr["is_reset"].sum() == 2 and len(tr["reward"]) >= 250


def test_oracle_quirks_cfg1_single():
    """Appendix A: fire persists across reset; robot_positions carries over while
    the reset observation is centred on [15, 15]; obs channel 0 is always 0."""
    tr = load("cfg1_single_traj")
    resets = np.nonzero(tr["is_reset"])[0]
    assert tr["fire_step"][resets[1]] > 0
    k = resets[1]
    assert tuple(tr["snap_view"][k]) == (15, 15)
    assert tuple(tr["snap_robots"][k][0]) == tuple(tr["snap_robots"][k - 1][0])
    assert np.all(tr["snap_obs"][:, ..., 0] == 0)
