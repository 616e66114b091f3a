"""Data-parallel training on the device, world size 2 (two processes sharing cuda:0, gloo
carrying the gradient all-reduce on device tensors -- RCCL cannot put two ranks on one GPU)
against the world-1 run (tests/dist_trainer_worker.py does the work in child processes):

* every env's state (global ids) after 8 training steps equals the world-1 run's: the
  sharding by global env id, the seeds and the act draws keyed by global agent id make
  trajectories independent of the GPU count;
* the trainer's online weights are bit-identical on both ranks after its learn steps;
* one learn step on each rank's half of a fixed union batch, with the hook averaging the
  gradients between backward and clip+Adam, equals one learn step on the whole union batch
  in one process: clipped gradients rtol 2e-4 (atol 1e-6 of their scale), norm rtol 1e-4,
  parameters within 1e-6 except where a near-zero gradient flips Adam's first-step sign.
Unmeasured on multi-GPU hardware: the RCCL path is the same hook on the "nccl" backend."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, out, mode="uniform"):
    port = _free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_trainer_worker.py"), str(r), str(world),
                               str(port), out, mode], env=env) for r in range(world)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs
    pre = "prio_" if mode == "prio" else ""
    return [dict(np.load(os.path.join(out, f"{pre}w{world}_r{r}.npz"))) for r in range(world)]


def test_world2_trainer_matches_world1(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = str(tmp_path)
    w1 = _run(1, out)[0]
    w2 = _run(2, out)
    E = w1["pos"].shape[0] // 2
    for r in range(2):
        for k in ["pos", "flags", "health", "acc", "rmap", "robots", "view", "scal", "py_mt", "np_mt"]:
            assert np.array_equal(w2[r][k], w1[k][r * E:(r + 1) * E]), (r, k)
    assert w2[0]["learn_steps"] >= 6
    assert np.array_equal(w2[0]["trainer_params"], w2[1]["trainer_params"])
    assert np.array_equal(w2[0]["learn_params"], w2[1]["learn_params"])
    assert np.array_equal(w2[0]["learn_grads"], w2[1]["learn_grads"])
    g1, g2 = w1["learn_grads"], w2[0]["learn_grads"]
    np.testing.assert_allclose(g2, g1, rtol=2e-4, atol=1e-6 * np.abs(g1).max())
    assert abs(w2[0]["learn_norm"] - w1["learn_norm"]) <= 1e-4 * w1["learn_norm"]
    # Adam's first step moves each weight by ~lr * sign(g): only near-zero gradients may flip
    diff = np.abs(w2[0]["learn_params"] - w1["learn_params"])
    assert (diff > 1e-6).mean() <= 1e-3 and diff.max() <= 2.1e-3, (diff.max(), (diff > 1e-6).mean())


def test_world2_prioritized_replay_cfg5_shape(tmp_path):
    """cfg5's multi-GPU shape on two ranks (gloo on one GPU): 32 robots per env, prioritized replay
    with one sum/min tree pair per rank over the rank's own ring, the gradient all-reduce hook.
    * env states by global id equal the world-1 run's (epsilon 1: actions do not depend on the
      weights), and both ranks hold bit-identical online weights after their learn steps;
    * every rank's trees are consistent with their leaves: each internal node is exactly the sum
      (min) of its children, the max leaf bounds every leaf, leaves beyond the ring's fill are 0;
    * the importance-weighted learn on each rank's half of a fixed union batch, averaged by the
      hook, equals the union-batch learn in one process (the tolerances above), and every row's
      |TD error| (the priorities' input) equals the world-1 row's within f32 rounding."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = str(tmp_path)
    w1 = _run(1, out, "prio")[0]
    w2 = _run(2, out, "prio")
    E = w1["pos"].shape[0] // 2
    for r in range(2):
        for k in ["pos", "flags", "health", "acc", "rmap", "robots", "view", "scal", "py_mt", "np_mt"]:
            assert np.array_equal(w2[r][k], w1[k][r * E:(r + 1) * E]), (r, k)
    assert w2[0]["learn_steps"] >= 6
    assert np.array_equal(w2[0]["trainer_params"], w2[1]["trainer_params"])
    for res in (w1, w2[0], w2[1]):
        ts, tm = res["tsum"], res["tmin"]
        C = ts.shape[0] // 2
        leaves = ts[C:]
        assert np.array_equal(ts[1:C], ts[2::2] + ts[3::2])
        assert np.array_equal(tm[1:C], np.minimum(tm[2::2], tm[3::2]))
        n = int(res["replay_size"])
        assert (leaves[:n] > 0).all() and (leaves[n:] == 0).all(), n
        assert res["max_leaf"][0] >= leaves.max() > 0
    assert not np.array_equal(w2[0]["tsum"], w2[1]["tsum"])  # each rank its own shard
    assert np.array_equal(w2[0]["learn_params"], w2[1]["learn_params"])
    g1, g2 = w1["learn_grads"], w2[0]["learn_grads"]
    np.testing.assert_allclose(g2, g1, rtol=2e-4, atol=1e-6 * np.abs(g1).max())
    assert abs(w2[0]["learn_norm"] - w1["learn_norm"]) <= 1e-4 * w1["learn_norm"]
    diff = np.abs(w2[0]["learn_params"] - w1["learn_params"])
    assert (diff > 1e-6).mean() <= 1e-3 and diff.max() <= 2.1e-3, (diff.max(), (diff > 1e-6).mean())
    td2 = np.concatenate([w2[0]["learn_td"], w2[1]["learn_td"]])
    np.testing.assert_allclose(td2, w1["learn_td"], rtol=1e-5, atol=1e-6 * np.abs(w1["learn_td"]).max())
