"""The CPU restatements of the build's counter-based draws (oracle/draw_oracle.c):
epsilon-greedy actions, uniform replay slots, the fused MLP's dropout hash.

Philox4x32-10 itself is pinned by its published known-answer vectors
(tests/test_prio_cpu.py); here: the restatements' laws (rates, ranges, windows, first
maximum) and agreement of the two independent host restatements of the dropout hash
(oracle C vs evacx.qmlp.dropout_keep numpy). The replay sampler draws without replacement
(a keyed Feistel permutation per learn step), as random.sample does. The GPU kernels are compared with these
index for index in tests/test_draws_gpu.py."""
import numpy as np
import pytest

from oracle import oracle as orc


def test_epsilon_greedy_argmax_first_maximum():
    Q = np.array([[0, 1, 3, 3, 2], [5, 5, 5, 5, 5], [-1, -2, -3, -4, -0.5]], np.float32)
    assert orc.epsilon_greedy(Q, 0.0, 1, 0).tolist() == [2, 0, 4]  # np.argmax semantics


def test_epsilon_greedy_rate_and_uniformity():
    n = 200000
    Q = np.zeros((n, 5), np.float32)
    Q[:, 3] = 1.0
    a = orc.epsilon_greedy(Q, 0.25, 7, 0)
    assert abs((a != 3).mean() - 0.25 * 0.8) < 0.005  # the random action is 3 one time in five
    a1 = orc.epsilon_greedy(Q, 1.0, 7, 0)
    counts = np.bincount(a1, minlength=5) / n
    assert np.all(np.abs(counts - 0.2) < 0.005), counts
    # counter-based: row i with offset o is row i + o with offset 0
    assert np.array_equal(orc.epsilon_greedy(Q[:1000], 0.5, 9, 300), orc.epsilon_greedy(Q[:1300], 0.5, 9, 0)[300:])


@pytest.mark.parametrize("base,size,cap", [(0, 1000, 1 << 12), (3000, 2000, 1 << 12), (0, 1 << 20, 1 << 20),
                                           (5, 3, 8), (0, 1, 4)])
def test_replay_indices_without_replacement(base, size, cap):
    """random.sample semantics (agents/dqn_agent.py:132): B <= size distinct slots of the window;
    B = size draws every slot once (a permutation of the window)."""
    B = min(size, 50000)
    idx = orc.replay_indices(base, size, cap, B, 11, 0)
    rel = (idx - base) % cap
    assert np.all((idx >= 0) & (idx < cap)) and np.all(rel < size)
    assert len(np.unique(idx)) == B
    full = orc.replay_indices(base, size, cap, size, 11, 0)
    assert np.array_equal(np.sort((full - base) % cap), np.arange(size))
    assert np.array_equal(full[:B], idx)  # a prefix of the step's permutation
    if size >= 1000:
        h = np.bincount((rel * 10) // size, minlength=10) / len(idx)
        assert np.all(np.abs(h - 0.1) < 0.01), h


def test_replay_indices_fresh_permutation_per_draw_and_stream():
    a = orc.replay_indices(0, 1 << 20, 1 << 20, 4096, 11, 0)
    b = orc.replay_indices(0, 1 << 20, 1 << 20, 4096, 11, 4096)
    c = orc.replay_indices(0, 1 << 20, 1 << 20, 4096, 11, 0, stream=3)
    d = orc.replay_indices(0, 1 << 20, 1 << 20, 4096, 12, 0)
    for x, y in ((a, b), (a, c), (a, d)):  # independent samples: overlap ~ B^2 / size = 16
        assert len(np.intersect1d(x, y)) < 64


def test_replay_indices_inclusion_is_uniform():
    """Over many learn steps (offsets) every slot is drawn with probability B / size, and the
    first draw is uniform -- what random.sample gives."""
    size, B, n = 37, 5, 20000
    inc = np.zeros(size)
    first = np.zeros(size)
    for o in range(n):
        idx = orc.replay_indices(0, size, 64, B, 3, o * B)
        assert len(np.unique(idx)) == B
        inc[idx] += 1
        first[idx[0]] += 1
    assert np.all(np.abs(inc / n - B / size) < 0.012), inc / n
    assert np.all(np.abs(first / n - 1 / size) < 0.006), first / n


@pytest.mark.parametrize("p", [0.2, 0.5])
def test_dropout_hash_two_restatements_agree(p):
    from evacx.qmlp import dropout_keep
    a = orc.dropout_keep(12345, 7, p, 301)
    b = dropout_keep(12345, 7, p, 301)
    assert np.array_equal(a.astype(bool), b)
    assert abs(a.mean() - (1 - p)) < 0.01
