"""Pin the prioritized-replay oracle (oracle/prio_oracle.c).

The reference has no prioritized replay (uniform random.sample over its deque,
Louvre_Evacuation/agents/dqn_agent.py:132), so parity with the reference is not
applicable here: the oracle is pinned by Philox4x32-10's published known-answer
vectors (Random123 kat_vectors), hand-computed segment-tree cases and the sampling
law of proportional prioritization (P(i) = p_i / sum p)."""
import numpy as np

from oracle import oracle as orc


def test_philox4x32_10_known_answers():
    kat = [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
         [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
    ]
    for ctr, key, want in kat:
        assert list(orc.philox4x32_10(ctr, key)) == want


def _u53(seed, k, offset=0):
    c = k + offset
    q = orc.philox4x32_10([c & 0xFFFFFFFF, c >> 32, 0x9E12A5, 0], [seed & 0xFFFFFFFF, seed >> 32])
    return ((int(q[0]) >> 5) * 67108864.0 + (int(q[1]) >> 6)) / 9007199254740992.0


def test_tree_known_answers():
    C = 1024
    t = orc.PrioTrees(C)
    assert t.max_leaf[0] == 1.0 and t.sum[1] == 0.0 and np.isinf(t.mn[1])
    t.set_range(1022, 4)  # wraps: slots 1022, 1023, 0, 1
    assert t.sum[1] == 4.0 and t.mn[1] == 1.0
    assert [t.sum[C + j] for j in (1022, 1023, 0, 1, 2)] == [1.0, 1.0, 1.0, 1.0, 0.0]
    t.update([1022, 1023, 0, 1], np.array([0.0, 1.0, 2.0, 3.0], np.float32), eps=0.5, alpha=1.0)
    assert t.sum[1] == 8.0 and t.mn[1] == 0.5 and t.max_leaf[0] == 3.5
    # internal nodes are left + right, roots of the halves
    assert t.sum[2] == 2.5 + 3.5 and t.sum[3] == 0.5 + 1.5
    # stratified descent: segment k covers mass [2k, 2k+2); cumulative order is slot 0, 1, ..., 1022, 1023
    seed = 42
    idx, w = t.sample(4, 0.5, seed, 0)
    cum = [(0, 2.5), (1, 6.0), (1022, 6.5), (1023, 8.0)]  # slot, end of its mass interval
    for k in range(4):
        u = (k + _u53(seed, k)) * (8.0 / 4)
        want = next(s for s, end in cum if u < end)
        assert idx[k] == want, (k, u)
        p = t.sum[C + want]
        assert w[k] == np.float32((p / 0.5) ** -0.5)
    # a later duplicate wins (sequential loop)
    t.update([5, 5, 5], np.array([9.0, 1.0, 4.0], np.float32), eps=0.0, alpha=1.0)
    assert t.sum[C + 5] == 4.0 and t.max_leaf[0] == 9.0


def test_hidden_slots_never_sampled_and_new_get_max():
    C = 2048
    t = orc.PrioTrees(C)
    t.set_range(0, 1500)
    rng = np.random.RandomState(1)
    t.update(np.arange(0, 1500, 3), rng.rand(500).astype(np.float32) * 5, eps=1e-6, alpha=0.6)
    t.set_range(1500, 300, 248)  # 300 new at max priority, slots 1800..2047 hidden
    assert np.all(t.sum[C + 1800:] == 0) and np.all(np.isinf(t.mn[C + 1800:]))
    assert np.all(t.sum[C + 1500:C + 1800] == t.max_leaf[0])
    idx, w = t.sample(4096, 0.4, 7, 0)
    assert idx.min() >= 0 and idx.max() < 1800
    assert np.all(w > 0) and np.all(w <= 1.0)
    assert np.all(np.diff(idx) >= 0)  # stratified: segments are in slot order


def test_sampling_law_is_proportional():
    C = 1024
    t = orc.PrioTrees(C)
    t.set_range(0, 64)
    pr = (np.arange(64) % 7 + 1).astype(np.float32)
    t.update(np.arange(64), pr, eps=0.0, alpha=1.0)
    counts = np.zeros(64)
    B = 1 << 14
    for s in range(8):
        idx, _ = t.sample(B, 1.0, 100 + s, 0)
        counts += np.bincount(idx, minlength=C)[:64]
    expect = pr / pr.sum() * counts.sum()
    # stratification makes the counts far tighter than multinomial: within 2 per pass
    assert np.all(np.abs(counts - expect) <= 16 + 1e-9), np.abs(counts - expect).max()
