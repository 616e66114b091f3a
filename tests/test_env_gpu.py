"""GPU parity of the HIP env path (libevacx.so) against the reference and the oracle.

* golden replays: the reference's own trajectories (tests/golden, captured by
  tools/capture_golden.py) re-run on the GPU from the recorded MT19937 states,
  bit-exact on every state field, observation, reward and done flag;
* oracle parity at scale: E independent envs per layout (36x30 P150 R1,
  64x64 P569 R8, 128x128 P2276 R16), seeds 1234+env, random actions,
  auto-reset, bit-exact against oracle/evac_oracle.c on every step.
"""
import numpy as np
import pytest
import torch

from golden_util import FIELDS, digest, load, traj_spec

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def fixture_tables(traj):
    from golden_util import traj_tables
    return traj_tables(traj)


def gpu_state_fields(env, e, obs64):
    st = env.host_state(e)
    return dict(pos=st["pos"], health=st["health"], acc=st["acc"], flags=st["flags"], rmap=st["rmap"],
                thmap=st["thmap"], robots=st["robots"], view=st["view"], obs=obs64[e]), st


@pytest.mark.parametrize("traj", ["cfg1_single_traj", "cfg1_multi_traj", "g64_multi_traj", "g128_multi_traj",
                                  "g128_long_traj"])
def test_gpu_replays_reference_trajectory(traj):
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    tables, P = fixture_tables(traj)
    tr = load(traj)
    E = 3  # identical copies: envs must not interfere
    lay = DeviceLayout(tables, P)
    env = VecEnv(lay, E, thmap=True)
    R = lay.R
    first = True
    for k in range(len(tr["reward"])):
        if tr["is_reset"][k]:
            if first:
                env.set_rng(np.tile(tr["rng_py"][k], (E, 1)), np.tile(tr["rng_np"][k], (E, 1)))
                first = False
            env.reset()
        else:
            a = torch.from_numpy(np.tile(tr["actions"][k].astype(np.int32), E)).cuda()
            env.step(a)
        obs64 = env.expand_obs(torch.float64).cpu().numpy()
        torch.cuda.synchronize()
        for e in range(E):
            f, st = gpu_state_fields(env, e, obs64)
            if k + 1 < len(tr["reward"]):
                assert np.array_equal(st["py_mt"], tr["rng_py"][k + 1]), (k, e, "py stream")
                assert np.array_equal(st["np_mt"], tr["rng_np"][k + 1]), (k, e, "np stream")
            for name in FIELDS:
                assert np.array_equal(digest(name, f[name]), tr["dig_" + name][k]), (k, e, name)
            assert int(st["scal"][0]) == tr["fire_step"][k]
            assert int(st["scal"][1]) == tr["cur_step"][k]
            if not tr["is_reset"][k]:
                assert env.reward[e].item() == tr["reward"][k], (k, e)
                assert bool(env.done[e].item()) == bool(tr["done"][k]), (k, e)
    env.check_err()
    py, nps = env.get_rng()
    assert np.array_equal(py[0], tr["rng_py_final"]) and np.array_equal(nps[0], tr["rng_np_final"])


def _oracle_pair(spec, P, E, steps, seed0=1234, act_seed=7, thmap=True, check_every=1, auto_reset=False,
                 wide=False):
    """Run E envs on the GPU and in the oracle with identical seeds/actions.
    auto_reset: finished envs are reset inside the step launch (VecEnv.step
    auto_reset); their terminal observations are checked from env.obs_term.
    wide: evx_env_order before every step, so envs with >= P/4 persons in play run
    their rows phase on a whole workgroup (rows_wide)."""
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables
    from oracle import oracle as orc
    tables = build_tables(spec)
    lay = DeviceLayout(tables, P)
    env = VecEnv(lay, E, thmap=thmap)
    R = spec.R
    env.seed([seed0 + i for i in range(E)])
    olay = orc.Layout.from_tables(tables, P)
    oenvs = [orc.Env(olay, thmap=thmap) for _ in range(E)]
    for i, oe in enumerate(oenvs):
        oe.seed(seed0 + i)
    env.reset()
    oobs = [oe.reset() for oe in oenvs]
    rng = np.random.RandomState(act_seed)
    n_resets = 0
    max_heavy = 0
    for s in range(steps + 1):
        if s > 0:
            acts = rng.randint(0, 5, size=(E, R)).astype(np.int32)
            acts[rng.rand(E, R) < 0.02] = 7  # invalid actions are ignored by the reference
            if wide:
                env.compute_order(force=True)
                max_heavy = max(max_heavy, int(env.order[E].item()))
            env.step(torch.from_numpy(acts.reshape(-1)).cuda(), order=not wide, auto_reset=auto_reset)
            res = [oe.step(acts[i]) for i, oe in enumerate(oenvs)]
            oobs = [r[0] for r in res]
            rew = env.reward.cpu().numpy()
            done = env.done.cpu().numpy().astype(bool)
            for i in range(E):
                assert rew[i] == res[i][1], (s, i, rew[i], res[i][1])
                assert done[i] == res[i][2], (s, i)
            if auto_reset and done.any():
                term = env.expand_obs(torch.float64, env.obs_term).cpu().numpy()
                for i in np.nonzero(done)[0]:
                    assert np.array_equal(term[i], oobs[i]), (s, i, "terminal obs")
                    oobs[i] = oenvs[i].reset()
                    n_resets += 1
        if s % check_every == 0 or s == steps:
            obs64 = env.expand_obs(torch.float64).cpu().numpy()
            obs32 = env.expand_obs(torch.float32).cpu().numpy()
            for i in range(E):
                f, st = gpu_state_fields(env, i, obs64)
                ost = oenvs[i].state()
                for name in ["pos", "health", "acc", "flags", "rmap", "robots", "view"]:
                    assert np.array_equal(f[name], ost[name]), (s, i, name)
                if thmap:
                    assert np.array_equal(f["thmap"], ost["thmap"]), (s, i, "thmap")
                assert np.array_equal(st["scal"], ost["scal"]), (s, i, "scal")
                assert np.array_equal(st["py_mt"], ost["py_mt"]), (s, i, "py_mt")
                assert np.array_equal(st["np_mt"], ost["np_mt"]), (s, i, "np_mt")
                assert np.array_equal(obs64[i], oobs[i]), (s, i, "obs")
                assert np.array_equal(obs32[i], oobs[i].astype(np.float32)), (s, i, "obs32")
        if s > 0 and not auto_reset:
            d = env.done.clone()
            if d.any():
                n_resets += int(d.sum())
                env.reset(mask=d)
                for i in np.nonzero(d.cpu().numpy())[0]:
                    oobs[i] = oenvs[i].reset()
    env.check_err()
    _oracle_pair.max_heavy = max_heavy
    return n_resets


def test_gpu_vs_oracle_cfg1_many_envs_with_resets():
    _need_gpu()
    from evacx.layout import reference_single
    n = _oracle_pair(reference_single(), 150, E=48, steps=260, check_every=13)
    assert n > 48  # every env went through several episodes (fire saturated)


def test_gpu_auto_reset_vs_oracle_cfg1():
    """Resets fused into the step launch: same states, observations and streams."""
    _need_gpu()
    from evacx.layout import reference_single
    n = _oracle_pair(reference_single(), 150, E=48, steps=260, check_every=13, auto_reset=True)
    assert n > 48


def test_gpu_auto_reset_vs_oracle_dense():
    _need_gpu()
    from evacx.layout import synthetic
    n = _oracle_pair(synthetic(24, 20, 4), 380, E=16, steps=120, check_every=3, auto_reset=True)
    assert n > 0


def test_gpu_wide_rows_vs_oracle_128_r16():
    """Heavy envs (rows phase on 4 waves) against the oracle at the benchmark layout."""
    _need_gpu()
    from evacx.layout import synthetic
    _oracle_pair(synthetic(128, 128, 16), 2276, E=6, steps=40, check_every=5, wide=True)
    assert _oracle_pair.max_heavy == 6


def test_gpu_wide_rows_vs_oracle_dense():
    """Wide and single-wave envs in one launch, big shuffles, episodes ending."""
    _need_gpu()
    from evacx.layout import synthetic
    _oracle_pair(synthetic(24, 20, 4), 380, E=16, steps=120, check_every=1, wide=True, auto_reset=True)
    assert _oracle_pair.max_heavy == 16


def test_gpu_wide_rows_vs_oracle_cfg1_resets():
    _need_gpu()
    from evacx.layout import reference_single
    n = _oracle_pair(reference_single(), 150, E=48, steps=260, check_every=13, wide=True, auto_reset=True)
    assert n > 48 and _oracle_pair.max_heavy > 0


def test_gpu_vs_oracle_multi_cfg1():
    _need_gpu()
    from evacx.layout import reference_multi
    _oracle_pair(reference_multi(), 150, E=16, steps=120, check_every=7)


def test_gpu_vs_oracle_synthetic_64():
    _need_gpu()
    from evacx.layout import synthetic
    _oracle_pair(synthetic(64, 64, 8), 569, E=12, steps=60, check_every=6)


def test_gpu_vs_oracle_synthetic_128_r16():
    _need_gpu()
    from evacx.layout import synthetic
    _oracle_pair(synthetic(128, 128, 16), 2276, E=6, steps=40, check_every=5)


def test_gpu_vs_oracle_dense_conflicts():
    """Many people on a small grid: heavy move conflicts, duplicates, big shuffles."""
    _need_gpu()
    from evacx.layout import synthetic
    _oracle_pair(synthetic(24, 20, 4), 380, E=16, steps=50, check_every=1)


def test_order_ahead_and_obs_double_buffer_do_not_change_results():
    """The lagged trainer's scheduling: the dispatch order computed one step ahead on
    another stream (racing the step that reads the other order buffer) and observations
    double-buffered. Same states bit for bit as the plain path; every order a permutation."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    lay = DeviceLayout(build_tables(synthetic(24, 20, 4)), 380)
    E = 300
    a = VecEnv(lay, E)
    b = VecEnv(lay, E, obs_buffers=2)
    for v in (a, b):
        v.seed([55 + i for i in range(E)])
        v.reset()
    side = torch.cuda.Stream()
    g = torch.Generator(device="cuda").manual_seed(3)
    for t in range(40):
        acts = torch.randint(0, 5, (E * lay.R,), device="cuda", dtype=torch.int32, generator=g)
        a.step(acts, auto_reset=True)
        prev = b.obs
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # overlaps b's step below
            b.compute_order(ahead=True)
        b.step(acts, order=False, auto_reset=True)
        torch.cuda.current_stream().wait_stream(side)
        assert b.obs_prev.data_ptr() == prev.data_ptr() and b.obs.data_ptr() != prev.data_ptr()
        torch.cuda.synchronize()
        ordr = b.order.cpu().numpy()
        assert np.array_equal(np.sort(ordr[:E]), np.arange(E)), t
        assert np.array_equal(a.obs.cpu().numpy(), b.obs.cpu().numpy()), t
        assert np.array_equal(a.obs_term.cpu().numpy(), b.obs_term.cpu().numpy()), t
        assert np.array_equal(a.reward.cpu().numpy(), b.reward.cpu().numpy()), t
    for name in ["pk", "health", "acc", "rmap", "scal", "py_mt", "np_mt"]:
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    a.check_err()
    b.check_err()


def test_gpu_vs_oracle_cfg4_256_single_robot():
    """BASELINE cfg4 geometry: 256x256 grid, 9102 people, one robot (two envs per
    workgroup: the layout's LDS does not fit four)."""
    _need_gpu()
    from evacx.layout import synthetic
    _oracle_pair(synthetic(256, 256, 1), 9102, E=3, steps=24, check_every=8, thmap=False)


def test_gpu_vs_oracle_cfg5_128_r32():
    """BASELINE cfg5 geometry: 128x128, 2276 people, 32 robots; heavy envs on 4 waves."""
    _need_gpu()
    from evacx.layout import synthetic
    _oracle_pair(synthetic(128, 128, 32), 2276, E=5, steps=30, check_every=6, wide=True, auto_reset=True)


def test_split_parts_on_two_streams_match_unsplit():
    """VecEnv.split: parts sharing the parent's storage, stepped concurrently on their own
    streams (the grouped trainer's schedule), give the unsplit env's results bit for bit;
    the parent still reads and resets all envs."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    lay = DeviceLayout(build_tables(synthetic(24, 20, 4)), 380)
    E = 512
    a = VecEnv(lay, E)
    b = VecEnv(lay, E, obs_buffers=2)
    for v in (a, b):
        v.seed([99 + i for i in range(E)])
        v.reset()
    parts = b.split(2)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    g = torch.Generator(device="cuda").manual_seed(5)
    k = (E // 2) * lay.R
    for t in range(30):
        acts = torch.randint(0, 5, (E * lay.R,), device="cuda", dtype=torch.int32, generator=g)
        a.step(acts, auto_reset=True)
        cur = torch.cuda.current_stream()
        for i, (p, s) in enumerate(zip(parts, streams)):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                p.step(acts[i * k:(i + 1) * k], auto_reset=True)
        for s in streams:
            cur.wait_stream(s)
        if t == 17:  # the parent resets across both parts
            m = torch.zeros(E, dtype=torch.bool, device="cuda")
            m[::7] = True
            a.reset(mask=m)
            b.reset(mask=m)
        torch.cuda.synchronize()
        assert torch.equal(a.obs, b.obs), t
        assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done), t
    for name in ["pk", "health", "acc", "rmap", "scal", "py_mt", "np_mt", "robots", "view"]:
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    st_a, st_b = a.host_state(300), b.host_state(300)
    assert all(np.array_equal(st_a[f], st_b[f]) for f in ["pos", "health", "acc"])
    b.check_err()


def test_heavy_and_light_parts_on_two_streams_match_one_launch():
    """evx_env_step_part: the heavy envs of the dispatch order (part 1) and the rest
    (part 2) stepped by two launches on two streams, concurrently, give the one-launch
    step's results bit for bit (fused resets included)."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    lay = DeviceLayout(build_tables(synthetic(24, 20, 4)), 380)
    E = 512
    a = VecEnv(lay, E)
    b = VecEnv(lay, E, obs_buffers=2)
    for v in (a, b):
        v.seed([71 + i for i in range(E)])
        v.reset()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.Generator(device="cuda").manual_seed(9)
    max_heavy = 0
    for t in range(40):
        acts = torch.randint(0, 5, (E * lay.R,), device="cuda", dtype=torch.int32, generator=g)
        a.step(acts, auto_reset=True)
        cur = torch.cuda.current_stream()
        b.compute_order()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            b.step(acts, order=False, auto_reset=True, part=1)
        with torch.cuda.stream(s2):
            b.step(acts, order=False, auto_reset=True, part=2)
        cur.wait_stream(s1)
        cur.wait_stream(s2)
        torch.cuda.synchronize()
        max_heavy = max(max_heavy, int(b.order[E].item()))
        assert torch.equal(a.obs, b.obs), t
        assert torch.equal(a.obs_term, b.obs_term), t
        assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done), t
    for name in ["pk", "health", "acc", "rmap", "scal", "py_mt", "np_mt", "robots", "view"]:
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert max_heavy > 0
    a.check_err()
    b.check_err()


@pytest.mark.parametrize("L,P,R,E", [(128, 2276, 16, 4096), (128, 2276, 16, 32768), (64, 569, 8, 4096)],
                         ids=["cfg3-4096", "cfg3-32768", "cfg2-4096"])
def test_stationary_mix_matches_oracle_at_bench_scale(L, P, R, E):
    """Parity where bench.py times: cfg3 (128x128, P 2276, R 16) at E envs -- 32768 is the bench
    workload (one-wave workgroups, env_step_kernel<1,false,false>), 4096 the 4-wave workgroups with
    the heavy-env path -- and cfg2 (64x64, P 569, R 8) at its bench size of 4096 envs, prepared
    exactly as bench.py --phase stationary does (1300 env-only steps, env g force-reset at
    preparation step g % 1200: env ages spread over an episode, saturated fire, heavy and light
    envs, fused auto-resets); then 64 envs spread over the age mix are snapshotted into the oracle
    and both step 100 more steps with the same actions -- every state field, MT stream, reward,
    done flag, observation and terminal observation (obs_term, on done) bit-exact on every step
    (the GPU steps all E envs with the heavy-first dispatch order, as in the bench).
    Reference: envs/evacuation_env.py:84-120 (_get_state), :122-172 (step), people.py:196-314."""
    _need_gpu()
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    from oracle import oracle as orc
    tables = build_tables(synthetic(L, L, R))
    lay = DeviceLayout(tables, P)
    env = VecEnv(lay, E)
    env.seed([1234 + i for i in range(E)])
    env.reset()
    gid = torch.arange(E, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(4321)
    acts = torch.empty(E * R, device="cuda", dtype=torch.int32)
    for w in range(1300):
        torch.randint(0, 5, (E * R,), device="cuda", dtype=torch.int32, generator=g, out=acts)
        env.step(acts, auto_reset=True)
        if w < 1200:
            env.reset(mask=(gid % 1200 == w) & ~env.done.bool())
    ids = list(range(0, E, E // 64))
    idt = torch.tensor(ids, device="cuda")
    olay = orc.Layout.from_tables(tables, P)
    oenvs = []
    for st in env.host_states(ids):
        oe = orc.Env(olay, thmap=False)
        oe.load_state(st)
        oenvs.append(oe)
    ages = np.array([oe.scal[1] for oe in oenvs])
    heavy0 = int(env.order[E].item()) if env.order is not None else 0
    assert ages.max() - ages.min() > 600, ages  # the sample spans the episode-age mix
    rng = np.random.RandomState(5)
    n_done = 0
    for s in range(100):
        a = rng.randint(0, 5, size=(E, R)).astype(np.int32)
        env.step(torch.from_numpy(a.reshape(-1)).cuda(), auto_reset=True)
        rew = env.reward[ids].cpu().numpy()
        dn = env.done[ids].cpu().numpy()
        ob = env.expand_obs(torch.float64, env.obs.view(E, -1)[idt].reshape(-1)).cpu().numpy()
        term = env.expand_obs(torch.float64, env.obs_term.view(E, -1)[idt].reshape(-1)).cpu().numpy() \
            if dn.any() else None
        sts = env.host_states(ids)
        for j, (e, oe) in enumerate(zip(ids, oenvs)):
            oobs, r, d = oe.step(a[e])
            assert rew[j] == r and bool(dn[j]) == d, (s, e, rew[j], r)
            if d:
                assert np.array_equal(term[j], oobs), (s, e, "terminal obs")
                oobs = oe.reset()
                n_done += 1
            assert np.array_equal(ob[j], oobs), (s, e, "obs")
            st = sts[j]
            for k in ["pos", "flags", "health", "acc", "rmap", "robots", "view", "scal", "py_mt", "np_mt"]:
                assert np.array_equal(st[k], getattr(oe, k)), (s, e, k)
    env.check_err()
    print(f"stationary mix {L}x{L} R{R} E{E}: ages {ages.min()}..{ages.max()}, heavy at start {heavy0}, "
          f"resets {n_done}")
